"""Parity cases shared by the golden-fixture generator and the tests.

Each case is a BASELINE.json configuration scaled so the CPU oracle finishes it in well under a second
(the full sizes are covered by the size-independent property tests in test_gpu_parity.py).
"""
from __future__ import annotations

from dataclasses import dataclass

from cudaraytracer_amd import abi, scenes


@dataclass(frozen=True)
class Case:
    name: str
    config: str
    width: int
    height: int
    spp: int
    depth: int | None = None  # None: the config's depth
    faithful_grid: bool = False
    rius_ltr: bool = False

    def cfg(self) -> scenes.Config:
        c = scenes.CONFIGS[self.config].scaled(self.width, self.height, self.spp)
        if self.depth is not None:
            c.depth = self.depth
        return c

    @property
    def flags(self) -> int:
        f = abi.RT_FLAG_FAITHFUL_GRID if self.faithful_grid else 0
        return f | (abi.RT_FLAG_RIUS_LEFT_TO_RIGHT if self.rius_ltr else 0)

    @property
    def rius_order(self) -> int:
        return 0 if self.rius_ltr else 1


CASES = [
    # BASELINE config 1 at full size with the reference's floor-division grid (Kernel.cu:184)
    Case("c1_full", "c1", 400, 225, 4, faithful_grid=True),
    Case("c2_rtiow_192x112_s16", "c2", 192, 112, 16),
    Case("c3_cornell_128_s16", "c3", 128, 128, 16),
    Case("c5_textured_160x96_s4", "c5", 160, 96, 4),
    Case("default_world_160x120_s8", "default", 160, 120, 8),
    Case("c2_rtiow_ltr_96x64_s8", "c2", 96, 64, 8, rius_ltr=True),
    Case("c2_rtiow_ragged_100x37_s4", "c2", 100, 37, 4),
]
CASE_BY_NAME = {c.name: c for c in CASES}

# Perf-mode RNG (RT_FLAG_RNG_PHILOX) fixtures: (case, frame index), seed 1984.
PHILOX_CASES = [(CASE_BY_NAME["c2_rtiow_ltr_96x64_s8"], 3), (CASE_BY_NAME["c3_cornell_128_s16"], 0)]
