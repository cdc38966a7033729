"""cProfile of the module engine's training loop with callers of the hot host calls (GPU box)."""
import cProfile
import io
import os
import pstats
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("WANDB_MODE", "dryrun")
import demo  # noqa: E402

pr = cProfile.Profile()
pr.enable()
demo.main(["--engine", "module", "--iters", "500", "--seed", "0", "--no_progress"])
pr.disable()
s = io.StringIO()
st = pstats.Stats(pr, stream=s).sort_stats("cumulative")
st.print_stats("runner.py|mlp.py|ddp.py|optim.py|gemm.py|_native.py|sampler.py|logging.py|module.py|autograd", 40)
st.print_callers("_cuda_getDeviceCount|run_backward|mse_loss")
print(s.getvalue())
