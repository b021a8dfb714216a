#!/usr/bin/env python3
"""Create an sqlite DB from a raw UniRef XML.gz (reference ``create_uniref_db.py``)."""
from proteinbert_pytorch_replication_amd.cli.etl import main_uniref_db

if __name__ == "__main__":
    main_uniref_db()
