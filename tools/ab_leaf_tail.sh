#!/bin/bash
# (records the A/B of a knob that is not in the product source)
# A/B of RT_TUNE_LEAF_TAIL (key 11: leave the leaf loop once <= K lanes still test primitives, the rest re-encoded as
# a leaf) against the tree before the knob (ab_src/render_base.hip = git show <parent>:...).  Parity of the knob
# build at K = 4 first (the golden cases through variant 3).  Same box, bench.py C2 / C3.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/ab_variants_build.sh base=ab_src/render_base.hip > gpurun_out/abbuild.log 2>&1 || exit 3
timeout -k 10 200 python - <<'PY' || exit 5
import sys; sys.path.insert(0, "tests"); sys.path.insert(0, ".")
import numpy as np, torch
from cases import CASES
from helpers import load_golden, digest
from cudaraytracer_amd import scenes
from cudaraytracer_amd._lib import lib
from cudaraytracer_amd.renderer import DeviceScene, Renderer
lib().rt_set_variant(3)
for K in (4, 16):
    lib().rt_set_tuning(11, K)
    for case in CASES:
        if case.faithful_grid: continue
        cfg = case.cfg(); g = load_golden(case.name)
        r = Renderer(cfg.width, cfg.height); r.render_init()
        r.render(DeviceScene(scenes.builtin(cfg.scene)), cfg.spp, cfg.depth, cfg.inputs(), flags=case.flags)
        torch.cuda.synchronize()
        assert np.array_equal(r.image(), g["pos"]), (K, case.name)
        assert digest(r.states()[:, :6]) == g["state_after_sha256"].tobytes(), (K, case.name)
print("leaf-tail parity ok")
PY
one() {  # lib label args
  RT_HIP_LIB=$1 timeout -k 10 200 python bench.py --no-cpu-baseline --no-philox-line --no-config-lines $3 > gpurun_out/ab.log 2>&1 || { tail -3 gpurun_out/ab.log; exit 4; }
  python -c "import json; d=json.loads(open('gpurun_out/ab.log').read().strip().splitlines()[-1]); print('$2', d['kernel_ms'], d['ms_per_step'])"
}
for r in 1 2; do
  one /tmp/ablib/base.so "c2 base" "--steps 20 --warmup 3"
  for K in 0 2 4 8 16; do one cudaraytracer_amd/librt_hip.so "c2 leaf_tail=$K" "--steps 20 --warmup 3 --tune 11=$K"; done
done
one /tmp/ablib/base.so "c3 base" "--config c3 --steps 2 --warmup 1"
for K in 0 4 16; do one cudaraytracer_amd/librt_hip.so "c3 leaf_tail=$K" "--config c3 --steps 2 --warmup 1 --tune 11=$K"; done
