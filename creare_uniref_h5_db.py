#!/usr/bin/env python3
"""Alias with the reference (misspelt) file name. Create the pretraining dataset store from the UniRef sqlite DB (reference ``creare_uniref_h5_db.py``)."""
from proteinbert_pytorch_replication_amd.cli.etl import main_uniref_h5

if __name__ == "__main__":
    main_uniref_h5()
