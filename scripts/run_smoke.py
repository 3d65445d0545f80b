"""__graft_entry__.smoke() without the build step (for GPU-box scripts: the
library is built in the build container and travels with the tree)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__  # noqa: E402

__graft_entry__.smoke()
