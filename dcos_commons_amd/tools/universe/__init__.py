"""Universe packaging: package identity, repositories and the stub-universe builder.

Reference: tools/universe/__init__.py.
"""
from dcos_commons_amd.tools.universe.package import Package, Version
from dcos_commons_amd.tools.universe.package_builder import UniversePackageBuilder, apply_template, sha256_of_file
from dcos_commons_amd.tools.universe.package_manager import (PackageManager, files_from_package, load_repository,
                                                             package_from_files, repo_tree_path)

__all__ = ["Package", "Version", "UniversePackageBuilder", "PackageManager", "apply_template", "sha256_of_file",
           "files_from_package", "load_repository", "package_from_files", "repo_tree_path"]
