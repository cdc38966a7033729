"""Metric logging with the reference's key names (``loss/lossX``, ``loss/lossY``,
``loss/loss``; ``demo.py:119-121``, ``demo_one_model_multi_gpu.py:129-130``).

Backends, chosen per run:
* wandb -- when importable and ``WANDB_MODE`` is not ``disabled``; ``--dry_run``
  sets ``WANDB_MODE=dryrun`` exactly like ``demo.py:160-161``;
* JSONL -- ``{log_dir}/metrics.jsonl``, always available (wandb is not installed
  on the MI355X image and the box has no network);
* stdout summaries.
Only rank 0 logs, as in the reference.
"""
from __future__ import annotations

import json
import math
import os
import time
from pathlib import Path


class MetricLogger:
    def __init__(self, project: str = "distributed tester", group: str = "base-demo", log_dir: str | None = None,
                 rank: int = 0, config: dict | None = None, use_wandb: bool | None = None):
        self.rank = rank
        self.enabled = rank == 0
        self._wandb = None
        self._f = None
        self.step = 0
        if not self.enabled:
            return
        mode = os.environ.get("WANDB_MODE", "")
        if use_wandb is None:
            use_wandb = mode != "disabled"
        if use_wandb:
            try:
                import wandb  # noqa: F401

                self._wandb = wandb.init(project=project, group=group, config=config or {},
                                         settings=wandb.Settings(start_method="thread"))
            except Exception:
                self._wandb = None
        if log_dir:
            Path(log_dir).mkdir(parents=True, exist_ok=True)
            self._f = open(Path(log_dir) / "metrics.jsonl", "a")
            self._f.write(json.dumps({"event": "start", "time": time.time(), "project": project, "group": group,
                                      "config": config or {}}) + "\n")

    @property
    def backend(self) -> str:
        if not self.enabled:
            return "none"
        return "+".join([b for b, on in (("wandb", self._wandb), ("jsonl", self._f)) if on]) or "stdout"

    def log(self, metrics: dict, step: int | None = None, commit: bool = True) -> None:
        if not self.enabled:
            return
        step = self.step if step is None else step
        if self._wandb is not None:
            self._wandb.log(metrics, step=step, commit=commit)
        if self._f is not None:
            self._f.write(json.dumps({"step": step, **{k: float(v) for k, v in metrics.items()}}) + "\n")
        if commit:
            self.step = step + 1

    def log_rows(self, steps: list[int], names: list[str], rows) -> None:
        """A block of per-step metrics in one call (the fused engines read their losses
        back once per launch): the same rows ``log`` writes -- one wandb row per step
        with every name, one JSONL line per step -- built as one string and written once.
        ``rows``: lists, or a host fp32 tensor [len(steps), len(names)] whose JSONL text
        the native formatter builds (``csrc/host_log.hip``, json.dumps' exact spelling)
        for consecutive steps."""
        if not self.enabled or not steps:
            return
        import torch

        if isinstance(rows, torch.Tensor):
            t = rows.detach()
            if (self._wandb is None and self._f is not None and t.device.type == "cpu" and t.dtype == torch.float32
                    and t.dim() == 2 and t.is_contiguous() and tuple(t.shape) == (len(steps), len(names))
                    and list(steps) == list(range(steps[0], steps[0] + len(steps)))):
                if self._write_native(steps[0], names, t):
                    self.step = steps[-1] + 1
                    return
            rows = t.tolist()
        if self._wandb is not None:
            for st, row in zip(steps, rows):
                self._wandb.log(dict(zip(names, map(float, row))), step=st)
        if self._f is not None:
            keys = [json.dumps(n) for n in names]

            def num(v):  # json.dumps' spelling (repr for finite floats, NaN / Infinity otherwise)
                v = float(v)
                return repr(v) if math.isfinite(v) else json.dumps(v)

            self._f.write("".join('{"step": %d, %s}\n' % (st, ", ".join("%s: %s" % (k, num(v)) for k, v in zip(keys, row)))
                                  for st, row in zip(steps, rows)))
        self.step = steps[-1] + 1

    def _write_native(self, step0: int, names, t) -> bool:
        import ctypes
        import json as _json

        from .. import _native as nat

        if not nat.native_enabled() or os.environ.get("DTP_NATIVE_LOG", "1") == "0":  # (A/B switch)
            return False
        lib = nat.load()
        keys = "".join(_json.dumps(k) + "\n" for k in names).encode()
        cap = lib.dtp_format_loss_rows_jsonl_bound(len(names), t.shape[0], len(keys))
        buf = ctypes.create_string_buffer(cap)
        m = lib.dtp_format_loss_rows_jsonl(t.data_ptr(), len(names), 0, t.shape[0], 1, step0, 1, keys, buf, cap)
        if m < 0:
            return False
        self._f.write(buf.raw[:m].decode("utf-8"))
        return True

    def finish(self) -> None:
        if not self.enabled:
            return
        if self._wandb is not None:
            try:
                self._wandb.finish()
            except Exception:
                pass
            self._wandb = None
        if self._f is not None:
            self._f.write(json.dumps({"event": "finish", "time": time.time()}) + "\n")
            self._f.close()
            self._f = None


def rank_print(rank: int, *msg) -> None:
    print(f"[Process {rank}]", *msg, flush=True)


class LossRing:
    """Per-step losses kept on the device, reduced across ranks and read back in chunks.

    The reference reduces each loss over gloo and logs it every iteration
    (``demo.py:114-121``), a host sync per step. Here ``put`` only queues device
    work (the row is chosen by a device-side slot counter, so ``put_device`` can sit
    inside a captured hipGraph); ``flush`` runs ONE all-reduce over the whole chunk
    and ONE device-to-host read, and returns the same per-step global means (sum
    over ranks / world). Every rank must call ``flush`` at the same steps (it is a
    collective).
    """

    def __init__(self, cap: int, width: int, device, world: int = 1, group=None):
        import torch

        self.buf = torch.zeros(cap, width, dtype=torch.float32, device=device)
        self.slot = torch.zeros(1, dtype=torch.int64, device=device)
        self.world = world
        self.group = group
        self.steps: list[int] = []
        self._inflight: list = []  # (event, pinned rows, steps) queued by flush(wait=False)

    def put_device(self, *values) -> None:
        """Device half of ``put`` (graph-capturable): row[slot] = values; slot += 1."""
        import torch

        row = torch.stack([v.detach().reshape(()).float() for v in values]).view(1, -1)
        self.buf.index_copy_(0, self.slot, row)
        self.slot.add_(1)

    def device_log(self):
        """``(rows, slot)`` for a kernel that writes the row itself (``MSELoss.pair(log=)``:
        the losses and the ring put in the loss's own launch instead of 3 more)."""
        return self.buf, self.slot

    def mark(self, step: int) -> None:
        """Host half of ``put``: the row just written holds ``step``."""
        self.steps.append(step)

    def put(self, step: int, *values) -> None:
        self.put_device(*values)
        self.mark(step)

    def full(self) -> bool:
        return len(self.steps) == self.buf.shape[0]

    def flush(self, wait: bool = True) -> list[tuple[int, list[float]]]:
        """Reduce the chunk and return the (step, values) rows that are on the host.
        ``wait=False`` (periodic flushes inside a run): the chunk's copy to pinned memory is
        only queued -- behind it the next steps' device work keeps the GPU busy -- and its
        rows come back from a later flush once the copy has arrived; ``wait=True``: every
        chunk, now.  Rows always come back in step order."""
        import torch

        if self.steps:
            from ..parallel import comm_util

            k = len(self.steps)
            chunk = self.buf[:k]
            comm_util.all_reduce_(chunk, self.group)
            ev = None
            if chunk.is_cuda:
                host = torch.empty(chunk.shape, dtype=chunk.dtype, pin_memory=True)
                host.copy_(chunk, non_blocking=True)  # stream-ordered before the rows are reused
                ev = torch.cuda.Event()
                ev.record()
            else:
                host = chunk.clone()
            self._inflight.append((ev, host, self.steps))
            self.steps = []
            self.slot.zero_()
        out = []
        while self._inflight and (wait or self._inflight[0][0] is None or self._inflight[0][0].query()):
            ev, host, steps = self._inflight.pop(0)
            if ev is not None:
                ev.synchronize()
            vals = host.tolist()
            if self.world > 1:
                vals = [[v / self.world for v in row] for row in vals]
            out.extend(zip(steps, vals))
        return out
