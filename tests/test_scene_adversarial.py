"""CPU: the adversarial scene of the flat-kernel exactness test is adversarial — on it the oracle's restatement of the
reference traversal (BVHNode::Hit with AABB::Hit culling, Hittable.cuh:387-439) and the brute-force closest hit over
all primitives render different pixels, so a kernel that returned the geometric closest hit would fail the GPU test
(tests/test_gpu_parity.py::test_flat_kernels_exact_on_ties_and_box_faces).  Also: the scene takes the flat path
(at most 16 primitives)."""
import numpy as np

from adversarial_scene import ADVERSARIAL_CONFIG, adversarial_scene
from oracle import py_oracle as po


def test_reference_culling_changes_pixels_in_the_adversarial_scene():
    cfg, sc = ADVERSARIAL_CONFIG, adversarial_scene()
    assert len(sc.hittables) <= 16
    imgs = []
    for exact in (False, True):
        st = po.init_states(cfg.width, cfg.height)
        img, _, _ = po.render(po.OracleScene(sc, exact=exact), cfg.width, cfg.height, cfg.spp, cfg.depth,
                              cfg.inputs(), st)
        imgs.append(img)
    differ = int((imgs[0] != imgs[1]).sum())
    assert differ > 100, differ
    assert len(np.unique(imgs[0])) > 1000  # the frame is not mostly sky


def test_reference_culling_changes_pixels_in_the_tiled_adversarial_scene():
    """The > 64-primitive variant (abutting floor tiles, an overlapping row) is adversarial too, and beyond the flat
    kernels' tables: the GPU test that renders it through LaunchKernel (tests/test_gpu_parity.py::
    test_launch_kernel_large_touching_scene_is_the_reference) runs the BVH kernels' exactness check and replay."""
    from adversarial_scene import adversarial_scene_tiled
    cfg, sc = ADVERSARIAL_CONFIG, adversarial_scene_tiled()
    assert len(sc.hittables) > 64
    imgs = []
    for exact in (False, True):
        st = po.init_states(cfg.width, cfg.height)
        img, _, _ = po.render(po.OracleScene(sc, exact=exact), cfg.width, cfg.height, cfg.spp, cfg.depth,
                              cfg.inputs(), st)
        imgs.append(img)
    differ = int((imgs[0] != imgs[1]).sum())
    assert differ > 50, differ
