"""``python -m wellflow.submit <model> columnNames columnTypes targetColumn storagePath [dataPath]``

Model names: cnn, mlp, mlp_online, lstm, gilbert (same argv contract as the per-model
scripts under "Artificial intelligence models/" and "Physical model/").
"""
import sys

from .train.job import run_job


def main(argv=None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    if not argv or argv[0] in ("-h", "--help"):
        print(__doc__)
        return 0
    run_job(argv[0], argv[1:])
    return 0


if __name__ == "__main__":
    sys.exit(main())
