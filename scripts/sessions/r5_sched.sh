#!/bin/bash
# round 5: LLVM scheduler strategy of mlp_train.hip (default build: max-ilp) against
# max-memory-clause (var_smc) and iterative-ilp (var_silp), K=2000 at batch 256 (split-batch)
# and 64 (4-lanes step), interleaved
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5sched
L=distributed_training_pytorch_amd/_lib
mkdir -p $O
for i in 1 2; do
  timeout -k 10 150 python bench.py --steps 2000 --warmup 200 >> $O/b256_main.json 2>> $O/err.log || exit $?
  for v in smc silp; do
    DTP_LIB=$L/var_$v/libdtp.so timeout -k 10 150 python bench.py --steps 2000 --warmup 200 >> $O/b256_$v.json 2>> $O/err.log || exit $?
  done
  timeout -k 10 150 python bench.py --steps 2000 --warmup 200 --scaling weak --batch 64 >> $O/b64_main.json 2>> $O/err.log || exit $?
  for v in smc silp; do
    DTP_LIB=$L/var_$v/libdtp.so timeout -k 10 150 python bench.py --steps 2000 --warmup 200 --scaling weak --batch 64 >> $O/b64_$v.json 2>> $O/err.log || exit $?
  done
done
