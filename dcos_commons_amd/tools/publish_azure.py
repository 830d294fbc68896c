"""``python -m dcos_commons_amd.tools.publish_azure <package> <universe dir> [artifacts...]``:
upload the artifacts and a stub universe to an Azure blob container (here: the emulated object
store).

As in the reference's tools/publish_azure.py, ``AZURE_STORAGE_ACCOUNT`` and
``AZURE_CONTAINER_NAME`` are mandatory (publishing fails without them, before anything is
rendered) and the blobs go to the container itself; the stub universe URL is the blob's URL
``https://<account>.blob.core.windows.net/<container>/<file>`` (what ``az storage blob url``
prints). ``AZURE_DIR_PATH`` optionally nests the blobs under a directory of the container.
After the upload the commands to (re)install from the new repository are logged, as the
reference prints them.
"""
from __future__ import annotations

import logging
import os
import sys
from typing import Sequence

from dcos_commons_amd.tools.publish_object_store import ObjectStorePublisher, main
from dcos_commons_amd.tools.universe.uploaders import AzureUploader

LOGGER = logging.getLogger(__name__)


def azure_directory_from_env() -> str:
    account = os.environ.get("AZURE_STORAGE_ACCOUNT", "")
    container = os.environ.get("AZURE_CONTAINER_NAME", "")
    if not account or not container:
        raise ValueError("It's mandatory to define the environment variables: "
                         "'AZURE_STORAGE_ACCOUNT' and 'AZURE_CONTAINER_NAME'")
    path = os.environ.get("AZURE_DIR_PATH", "").strip("/")
    url = f"https://{account}.blob.core.windows.net/{container}"
    return f"{url}/{path}" if path else url


class AzurePublisher(ObjectStorePublisher):
    def upload(self, work_dir: str = None) -> str:
        url = super().upload(work_dir)
        LOGGER.info("(Re)install your package using the following commands:\n"
                    "dcos package uninstall %s\ndcos package repo remove %s-azure\n"
                    "dcos package repo add --index=0 %s-azure '%s'\ndcos package install --yes %s",
                    self._name, self._name, self._name, url, self._name)
        return url


def azure_publisher(package_name: str, package_version: str, input_dir_path: str,
                    artifact_paths: Sequence[str]) -> AzurePublisher:
    dry = bool(os.environ.get("DRY_RUN"))
    return AzurePublisher(package_name, package_version, input_dir_path, artifact_paths,
                          AzureUploader(azure_directory_from_env(), dry), dry)


if __name__ == "__main__":
    sys.exit(main(sys.argv, azure_publisher))
