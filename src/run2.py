"""P2P smoke test, rank 1 (ref src/run2.py).  Start run1.py on the master (or locally)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from p2p import main  # noqa: E402

if __name__ == "__main__":
    sys.exit(main(1))
