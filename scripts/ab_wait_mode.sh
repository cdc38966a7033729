# Interleaved A/B of the host wait mode on the K=20 bench (GPU box): 8 runs each
mkdir -p gpurun_out
for i in 1 2 3 4 5 6 7 8; do
  for m in auto spin; do
    r=$(DTP_WAIT_MODE=$m timeout 60 python bench.py --steps 20 --warmup 5 2>/dev/null | grep '^{' | python3 -c "import json,sys; print(json.loads(sys.stdin.read())['ms_per_step']*1e3)") || exit 1
    echo "$m $r"
  done
done
