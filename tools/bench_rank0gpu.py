"""bench.py with every rank on cuda:0 (LOCAL_RANK forced to 0): the N>1 rehearsal on a
one-GPU box (tools/gpu_multi_rehearsal.sh)."""
import os
import runpy
import sys

os.environ["LOCAL_RANK"] = "0"
sys.argv[0] = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "bench.py")
runpy.run_path(sys.argv[0], run_name="__main__")
