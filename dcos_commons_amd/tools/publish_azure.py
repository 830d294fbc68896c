"""``python -m dcos_commons_amd.tools.publish_azure <package> <universe dir> [artifacts...]``
(reference: tools/publish_azure.py): publish to an Azure blob container (the emulated object store)."""
import sys

from dcos_commons_amd.tools.publish_object_store import azure_publisher, main

if __name__ == "__main__":
    sys.exit(main(sys.argv, azure_publisher))
