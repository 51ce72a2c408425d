"""P2P smoke test, rank 0 (ref src/run1.py).  Start run2.py on the peer (or locally)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from p2p import main  # noqa: E402

if __name__ == "__main__":
    sys.exit(main(0))
