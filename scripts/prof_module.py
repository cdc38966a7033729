"""Host-side profile of the module engine (demo.py --engine module): cProfile of the
whole run, top entries by cumulative and by own time."""
import cProfile
import pstats
import runpy
import sys

iters = sys.argv[1] if len(sys.argv) > 1 else "2000"
sys.argv = ["demo.py", "--engine", "module", "--iters", iters, "--seed", "0", "--no_progress"]
cProfile.run('runpy.run_path("demo.py", run_name="__main__")', "gpurun_out/module.prof")
st = pstats.Stats("gpurun_out/module.prof")
st.sort_stats("cumtime").print_stats(45)
st.sort_stats("tottime").print_stats(25)
