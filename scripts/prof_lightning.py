"""Host-side profile of the Lightning demo's module path (Trainer without the fused
engine): cProfile of a run, top entries by own time and by cumulative time."""
import cProfile
import pstats
import runpy
import sys

steps = sys.argv[1] if len(sys.argv) > 1 else "3000"
sys.argv = ["demo_pytorch_lightning.py", "--gpus", "1", "--steps", steps, "--seed", "0", "--root_dir", "/tmp/ltp",
            "--engine", "module"]
cProfile.run('runpy.run_path("demo_pytorch_lightning.py", run_name="__main__")', "gpurun_out/lt_module.prof")
st = pstats.Stats("gpurun_out/lt_module.prof")
st.sort_stats("tottime").print_stats(35)
st.sort_stats("cumtime").print_stats(60)
