"""``python -m dcos_commons_amd.tools.publish_aws <package> <universe dir> [artifacts...]``:
upload the artifacts and a stub universe to S3 (here: the emulated object store).

Destination, as in the reference's tools/publish_aws.py (``s3_urls_from_env``):

* ``S3_BUCKET`` (default ``infinity-artifacts``), ``S3_DIR_PATH`` (default ``autodelete7d``) and
  ``S3_DIR_NAME`` (default ``<timestamp>-<16 random characters>``) give
  ``s3://<bucket>/<dir path>/<package>/<dir name>``; ``S3_URL`` overrides that URL outright;
* ``ARTIFACT_DIR`` overrides the HTTP directory the universe links artifacts from (default
  ``https://<bucket>.s3.amazonaws.com/<dir path>/<package>/<dir name>``; with the emulated store,
  its HTTP address of the same bucket path);
* ``DRY_RUN`` renders without uploading.
"""
from __future__ import annotations

import os
import sys
from typing import Sequence, Tuple

from dcos_commons_amd.tools.publish_object_store import ObjectStorePublisher, main, unique_dir_name
from dcos_commons_amd.tools.universe.uploaders import S3Uploader, parse_s3_url


def s3_urls_from_env(package_name: str) -> Tuple[str, str]:
    """(S3 directory URL, HTTP directory URL or "" for the store's own address)."""
    bucket = os.environ.get("S3_BUCKET") or "infinity-artifacts"
    dir_path = (os.environ.get("S3_DIR_PATH") or "autodelete7d").strip("/")
    dir_name = os.environ.get("S3_DIR_NAME") or unique_dir_name()
    s3_url = os.environ.get("S3_URL") or f"s3://{bucket}/{dir_path}/{package_name}/{dir_name}"
    parse_s3_url(s3_url)   # fails early on a malformed override
    return s3_url.rstrip("/"), os.environ.get("ARTIFACT_DIR", "").rstrip("/")


class _S3Uploader(S3Uploader):
    """An S3 uploader whose HTTP directory can be overridden (``ARTIFACT_DIR``)."""

    def __init__(self, s3_directory: str, http_directory: str, dry_run: bool):
        super().__init__(s3_directory, dry_run)
        self._http_override = http_directory

    def http_directory_url(self) -> str:
        return self._http_override or super().http_directory_url()


def aws_publisher(package_name: str, package_version: str, input_dir_path: str,
                  artifact_paths: Sequence[str]) -> ObjectStorePublisher:
    dry = bool(os.environ.get("DRY_RUN"))
    s3_dir, http_dir = s3_urls_from_env(package_name)
    return ObjectStorePublisher(package_name, package_version, input_dir_path, artifact_paths,
                                _S3Uploader(s3_dir, http_dir, dry), dry)


if __name__ == "__main__":
    sys.exit(main(sys.argv, aws_publisher))
