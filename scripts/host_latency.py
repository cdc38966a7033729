"""Host-side launch + completion latency on this box: median over 200 round trips of a
1-element fill followed by synchronize, and of the same with 20 fills queued, plus the
load average (the K=20 bench line is dominated by these when they are slow)."""
import os
import statistics
import time

import torch

dev = torch.device("cuda", 0)
x = torch.zeros(1, device=dev)
torch.cuda.synchronize()


def rt(n):
    ts = []
    for _ in range(200):
        t0 = time.perf_counter()
        for _ in range(n):
            x.fill_(1.0)
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    return statistics.median(ts) * 1e6, max(ts) * 1e6


for n in (1, 20):
    med, mx = rt(n)
    print(f"{n} fill(s) + synchronize: median {med:.1f} us, max {mx:.1f} us")
print("loadavg", os.getloadavg(), "cpus", os.cpu_count())
