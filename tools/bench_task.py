"""Run the repository's bench.py in-process from the tree this file belongs to (so tools/xab.sh
can A/B bench.py configurations across two trees: tools/ and _abbase/tools/).

    python tools/bench_task.py --batch-per-gpu 512 --steps 20 --warmup 5"""

import os
import sys

root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, root)
sys.argv = [os.path.join(root, "bench.py")] + sys.argv[1:]

import bench  # noqa: E402

if __name__ == "__main__":
    bench.main()
