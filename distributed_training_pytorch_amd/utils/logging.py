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
