"""Save CI's ``stub-universe.properties`` next to the published package (reference:
tools/save_properties.py, which runs ``aws s3 cp`` from Jenkins' ``$WORKSPACE``).

``python -m dcos_commons_amd.tools.save_properties s3://<bucket>/<dir>`` uploads
``$WORKSPACE/stub-universe.properties`` through the S3 uploader (the emulated object store).
"""
from __future__ import annotations

import logging
import os
import sys

from dcos_commons_amd.tools.universe.uploaders import S3Uploader

LOGGER = logging.getLogger(__name__)
PROPERTIES_FILE_NAME = "stub-universe.properties"


def upload_to_s3(s3_dir_uri: str) -> str:
    path = os.path.join(os.environ.get("WORKSPACE", ""), PROPERTIES_FILE_NAME)
    if not os.path.isfile(path):
        raise FileNotFoundError(f"Could not find properties file: {path}")
    return S3Uploader(s3_dir_uri).upload(path, content_type="text/plain")


def main(argv) -> int:
    if len(argv) != 2:
        LOGGER.error("Syntax: %s s3://bucket/path/to/dir", argv[0])
        return 1
    upload_to_s3(argv[1])
    return 0


if __name__ == "__main__":
    logging.basicConfig(level=logging.INFO, format="%(message)s")
    sys.exit(main(sys.argv))
