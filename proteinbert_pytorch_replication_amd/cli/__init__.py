"""Command-line entry points: ``python -m proteinbert_pytorch_replication_amd.cli <command>``.

Commands: ``create-uniref-db`` (reference ``create_uniref_db.py``, C1), ``create-uniref-h5-db``
(reference ``creare_uniref_h5_db.py``, C2), ``pretrain`` and ``finetune``.
"""
