# """Dynamic (online, streaming) ANN flow-prediction model"""
# Usage :  python3 *columnNames *columnTypes targetColumn storagePath [dataPath] [--options]
# Submission entrypoint with the reference's argv contract (cnn.py:1-2, 41-44); the job
# runs on the wellflow MI355X engine (one process per GPU under torchrun, RCCL over xGMI).
import os
import sys

_here = os.path.dirname(os.path.abspath(__file__))
while _here != os.path.dirname(_here) and not os.path.isdir(os.path.join(_here, "wellflow")):
    _here = os.path.dirname(_here)
sys.path.insert(0, _here)

from wellflow.train.job import main  # noqa: E402

if __name__ == "__main__":
    sys.exit(main("mlp_online"))
