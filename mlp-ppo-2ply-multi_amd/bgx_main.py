#!/usr/bin/env python3
"""Run the reference's training entry point (src/main.py) on the MI355X engine.

    python mlp-ppo-2ply-multi_amd/bgx_main.py /path/to/reference/src/main.py

`python src/main.py` puts the script's own directory (src/) at the head of
sys.path, ahead of PYTHONPATH, so `from multi import ...` (main.py:2) would
load the reference's CPU workers. This launcher instead puts this package
first and the reference's src/ second, then runs main.py as __main__
(runpy.run_path adds nothing to sys.path for a file): main.py's own
`multiprocessing.set_start_method("spawn")` and its 7 worker processes
(main.py:86-91) inherit that sys.path, so every process imports this build's
multi / environments packages, and the reference's agents / utils / config
for the rest. Worker i drives an engine on GPU i; ids past the visible GPUs
idle (multi/worker.py).
"""
import os
import runpy
import sys

PKG = os.path.dirname(os.path.abspath(__file__))


def main(argv):
    if len(argv) < 2 or not argv[1].endswith(".py"):
        print(__doc__.strip().splitlines()[2].strip(), file=sys.stderr)
        return 2
    script = os.path.abspath(argv[1])
    src = os.path.dirname(script)
    sys.path[:0] = [PKG, src]
    sys.argv = [script] + argv[2:]
    runpy.run_path(script, run_name="__main__")
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv))
