"""Comparison helpers for RGBA8 images (tolerance contract of SURVEY.md §8(c) C3)."""
from __future__ import annotations

import hashlib
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def rgb(img: np.ndarray) -> np.ndarray:
    return np.ascontiguousarray(img).view(np.uint8).reshape(-1, 4)[:, :3].astype(np.int32)


def image_stats(a: np.ndarray, b: np.ndarray) -> dict:
    d = rgb(a) - rgb(b)
    ad = np.abs(d)
    return {
        "exact": float(np.mean(np.all(ad == 0, axis=1))),
        "within1": float(np.mean(np.all(ad <= 1, axis=1))),
        "within2": float(np.mean(np.all(ad <= 2, axis=1))),
        "mean_abs": float(ad.mean()),
        "mean_signed": float(d.mean()),
        "max": int(ad.max()) if ad.size else 0,
    }


def assert_tolerance_contract(a: np.ndarray, b: np.ndarray) -> dict:
    """SURVEY.md §8(c) C3 statistical contract (used where bit-exactness is not claimed)."""
    s = image_stats(a, b)
    assert s["within1"] >= 0.95 and s["within2"] >= 0.97, s
    assert s["mean_abs"] <= 0.3 and abs(s["mean_signed"]) <= 0.05, s
    return s


def digest(a: np.ndarray) -> bytes:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).digest()


def load_golden(name: str) -> dict:
    with np.load(os.path.join(GOLDEN, f"{name}.npz")) as z:
        return {k: z[k] for k in z.files}
