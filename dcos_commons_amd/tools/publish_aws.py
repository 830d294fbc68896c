"""``python -m dcos_commons_amd.tools.publish_aws <package> <universe dir> [artifacts...]``
(reference: tools/publish_aws.py): publish to an S3 bucket (the emulated object store)."""
import sys

from dcos_commons_amd.tools.publish_object_store import aws_publisher, main

if __name__ == "__main__":
    sys.exit(main(sys.argv, aws_publisher))
