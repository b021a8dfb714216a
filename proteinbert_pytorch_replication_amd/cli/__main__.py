"""``python -m proteinbert_pytorch_replication_amd.cli <command> [args]``."""
import sys

COMMANDS = {
    "create-uniref-db": ("etl", "main_uniref_db"),
    "create-uniref-h5-db": ("etl", "main_uniref_h5"),
    "pretrain": ("train", "pretrain_main"),
    "finetune": ("train", "finetune_main"),
    "dummy-tests": ("dummy_tests", "main"),
}


def main(argv=None) -> None:
    argv = list(sys.argv[1:] if argv is None else argv)
    if not argv or argv[0] not in COMMANDS:
        print("usage: python -m proteinbert_pytorch_replication_amd.cli {%s} [args]" % ",".join(COMMANDS))
        sys.exit(0 if argv and argv[0] in ("-h", "--help") else 2)
    mod, fn = COMMANDS[argv[0]]
    import importlib
    getattr(importlib.import_module(f"proteinbert_pytorch_replication_amd.cli.{mod}"), fn)(argv[1:])


if __name__ == "__main__":
    main()
