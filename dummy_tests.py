#!/usr/bin/env python3
"""Smoke pretraining driver (reference ``ProteinBERT/dummy_tests.py``); see ``--help``."""
from proteinbert_pytorch_replication_amd.cli.dummy_tests import main

if __name__ == "__main__":
    main()
