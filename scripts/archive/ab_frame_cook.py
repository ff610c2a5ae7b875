"""scripts/bench_frame.py --cook dev (framing + encode + cook of one 65,536-group
batch into device memory) with no CPU baseline: the A/B workload for
scripts/gpu_ab_kernels.sh, which passes no arguments."""
import os
import runpy
import sys

here = os.path.dirname(os.path.abspath(__file__))
sys.argv = [os.path.join(here, "bench_frame.py"), "--cook", "dev", "--cpu-sample", "0"]
runpy.run_path(sys.argv[0], run_name="__main__")
