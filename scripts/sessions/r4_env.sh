#!/bin/bash
# round 4: runtime knobs for the driver's K=20 line, fresh processes, interleaved:
#   intr0   HSA completion signals polled instead of interrupt-driven (HSA_ENABLE_INTERRUPT=0)
#   kernarg kernel arguments in device memory (HIP_FORCE_DEV_KERNARG=1)
#   active  the host spins on a completion signal up to 1 ms before sleeping (ROC_ACTIVE_WAIT_TIMEOUT=1000)
export TMPDIR=/tmp
D=${1:-r4env}
mkdir -p gpurun_out/$D
bash scripts/gpu_steps.sh \
  "400|$D/k20|for r in 1 2 3 4; do for v in none intr0 kernarg active; do case \$v in none) E=\"\";; intr0) E=\"HSA_ENABLE_INTERRUPT=0\";; kernarg) E=\"HIP_FORCE_DEV_KERNARG=1\";; active) E=\"ROC_ACTIVE_WAIT_TIMEOUT=1000\";; esac; echo \"env=\$v\"; env \$E python bench.py --steps 20 --warmup 5; done; done"
