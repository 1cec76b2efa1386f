"""In-process driver for kernel-trace A/Bs of the config-4 step: bench.py --workload train
--steps 4 --warmup 2 (no CPU baseline), run as __main__ in this process."""
import os
import runpy
import sys

root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, root)
os.chdir(root)
sys.argv = ["bench.py", "--workload", "train", "--steps", "4", "--warmup", "2", "--cpu-baseline", "0"]
runpy.run_path(os.path.join(root, "bench.py"), run_name="__main__")
