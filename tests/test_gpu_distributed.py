"""GPU test of the multi-rank bench path's RCCL leg (cudaraytracer_amd.parallel.BandGather over the `nccl` backend =
RCCL on ROCm).  The one-GPU box cannot host two RCCL ranks (RCCL refuses two ranks on one device), so this runs a
one-rank RCCL group in a child process: the pipelined gather — an asynchronous collective on RCCL's stream, the
render stream waiting for frame k's gather only after frame k + 1's render is enqueued — must return every frame
exactly as rendered.  The N > 1 exchange itself is covered by the gloo tests (tests/test_distributed.py) and runs
in the driver's 8-GPU scaling bench."""
from __future__ import annotations

import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import os, sys
sys.path.insert(0, sys.argv[1])
import numpy as np, torch, torch.distributed as dist
from cudaraytracer_amd import parallel, scenes
from cudaraytracer_amd.renderer import DeviceScene, Renderer
torch.cuda.set_device(0)
parallel.init_process_group("nccl")
assert dist.get_backend() == "nccl" and dist.get_world_size() == 1
cfg = scenes.CONFIGS["c2"].scaled(160, 97, 2)
ds = DeviceScene(scenes.builtin(cfg.scene))
band = parallel.DEFAULT_BAND_ROWS
r = Renderer(cfg.width, cfg.height, band_rows=band)
r.render_init()
g = parallel.BandGather(cfg.width, cfg.height, band)
expect, got = [], []
for k in range(4):
    r.render(ds, cfg.spp, cfg.depth, cfg.inputs())
    expect.append(r.pos.clone())   # (same stream: a copy of frame k before frame k + 1 overwrites r.pos)
    if k:
        got.append(g.finish().clone())  # frame k - 1, finished after frame k's render was enqueued
    g.start(r.pos)
got.append(g.finish().clone())
torch.cuda.synchronize()
for k in range(4):
    e = expect[k].view(cfg.height, cfg.width)
    assert torch.equal(got[k], e), k
    assert k == 0 or not torch.equal(expect[k], expect[k - 1])  # the frames differ (advancing RNG states)
dist.destroy_process_group()
print("pipelined rccl gather ok")
"""


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_pipelined_rccl_gather_returns_every_frame():
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), RANK="0", WORLD_SIZE="1",
               LOCAL_RANK="0")
    out = subprocess.run([sys.executable, "-c", CHILD, ROOT], env=env, capture_output=True, text=True, timeout=240)
    assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-4000:]
    assert "pipelined rccl gather ok" in out.stdout
