set -u
one() {  # label args
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-philox-line --no-config-lines $2 > gpurun_out/ab.log 2>&1 || { tail -3 gpurun_out/ab.log; exit 4; }
  python -c "import json; d=json.loads(open('gpurun_out/ab.log').read().strip().splitlines()[-1]); print('$1', d['kernel_ms'], d['ms_per_step'], flush=True)"
}
for r in 1 2 3; do
  for w in 3 4 5; do
    one "c5 pflat waves $w" "--config c5 --steps 40 --warmup 4 --tune 2=$w"
    one "c5 pflat philox waves $w" "--config c5 --steps 40 --warmup 4 --tune 2=$w --rng philox"
  done
done
timeout -k 10 400 python -u tools/flat_sweep.py --configs c1,default,c5,c3 --trips 2,3,4,6,8 --rounds 3
