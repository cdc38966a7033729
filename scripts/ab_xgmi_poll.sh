# Interleaved A/B of the in-kernel xGMI poll loop (GPU box): default build (pipelined polls)
# vs _lib/var_pollold (poll, wait, check, sleep), 2- and 8-rank one-GPU rehearsals.
set -o pipefail
mkdir -p gpurun_out
old="$(pwd)/distributed_training_pytorch_amd/_lib/var_pollold/libdtp.so"
for rep in 1 2 3; do
  for v in new old; do
    if [ "$v" = old ]; then export DTP_LIB="$old"; else unset DTP_LIB; fi
    for args in "" "--steps 20 --warmup 5"; do
      out=$(bash scripts/rehearse_share_gpu.sh "2 8" "$args") || { echo "$out"; exit 1; }
      echo "$v [${args:-K=2000}] $(echo $out | tr '\n' ' ')"
    done
  done
done
