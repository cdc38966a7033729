"""cProfile of the layer-split demo's loop (GPU box): where the host time goes."""
import cProfile
import io
import os
import pstats
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("WANDB_MODE", "dryrun")
import demo_one_model_multi_gpu as demo  # noqa: E402

pr = cProfile.Profile()
pr.enable()
demo.main(["--allow_shared_gpu", "--iters", "500", "--seed", "0", "--no_progress"])
pr.disable()
s = io.StringIO()
st = pstats.Stats(pr, stream=s).sort_stats("tottime")
st.print_stats(30)
st.print_callers("_cuda_getDeviceCount|is_available")
print(s.getvalue())
