# Driver-shaped headline (--steps 20 --warmup 5) vs the untimed clock prewarm
# length, alternating, extras off.
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2 3; do
  for pw in 0.25 1.0 2.0; do
    timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 --no-extras --no-cpu --prewarm-s $pw \
      > gpurun_out/pw_${pw}_${rep}.log 2>&1 || exit 99
    echo "pw=$pw rep=$rep $(grep '^{' gpurun_out/pw_${pw}_${rep}.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["kernel_us"], d["roofline"]["frac"])')" | tee -a gpurun_out/prewarm.txt
  done
done
