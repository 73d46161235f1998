"""A small scene built against the flat kernels' exactness check (render.hip flat_trace): coplanar rectangles that
overlap (exact ties in t over an area) and abut (shared edges), a floor and a wall meeting the rectangles' edges,
spheres tangent to the rectangles' plane whose box faces lie on the floor and wall planes, and a mirror sphere.
Used by tests/test_gpu_parity.py::test_flat_kernels_exact_on_ties_and_box_faces and pinned as adversarial (the
reference's box culling changes pixels against the brute-force closest hit) by tests/test_scene_adversarial.py."""
from cudaraytracer_amd import abi, scenes

# 160x120, 8 spp, depth 6, looking down -z at the z = 0 plane from 6 units
ADVERSARIAL_CONFIG = scenes.Config("adversarial", scenes.SCENE_THREE_SPHERES, 160, 120, 8, 6, (0.3, 0.2, 6.0),
                                   (0.0, 0.0, -1.0), 50.0)

_RECTS = [  # (type, centre, width, height, material)
    (abi.RT_XYRECT, (0.0, 0.0, 0.0), 2.0, 2.0, 0),   # x -1..1, y -1..1 on z = 0
    (abi.RT_XYRECT, (1.0, 0.5, 0.0), 2.0, 2.0, 1),   # the same plane, overlapping rect 0: ties in t
    (abi.RT_XYRECT, (2.0, 0.0, 0.0), 2.0, 2.0, 2),   # abutting rect 0 along x = 1
    (abi.RT_XZRECT, (0.0, -1.0, 1.0), 6.0, 6.0, 3),  # floor y = -1 along the rectangles' lower edges
    (abi.RT_YZRECT, (-1.0, 0.0, 1.0), 4.0, 4.0, 4),  # wall x = -1 along rect 0's left edge
]
_SPHERES = [((0.0, 0.0, 1.0), 1.0, 5),       # tangent to z = 0; box face z = 0 on the rectangles' plane
            ((-0.5, -0.5, 0.5), 0.5, 6),     # box faces on the floor, the wall and z = 0
            ((1.5, 0.5, 0.75), 0.75, 7)]     # mirror, tangent to z = 0
_COLOURS = [(0.8, 0.2, 0.2), (0.2, 0.8, 0.2), (0.2, 0.2, 0.8), (0.7, 0.7, 0.7), (0.6, 0.5, 0.3), (0.9, 0.9, 0.2),
            (0.3, 0.9, 0.9), (0.8, 0.8, 0.8)]


def adversarial_scene() -> scenes.Scene:
    n = len(_RECTS) + len(_SPHERES)
    h = (abi.HittableDesc * n)()
    m = (abi.MaterialDesc * len(_COLOURS))()
    for i, (t, c, w, hh, mat) in enumerate(_RECTS):
        h[i].type, h[i].is_active, h[i].material = t, 1, mat
        h[i].center[:] = list(c)
        h[i].width, h[i].height = w, hh
    for j, (c, r, mat) in enumerate(_SPHERES):
        i = len(_RECTS) + j
        h[i].type, h[i].is_active, h[i].material, h[i].radius = abi.RT_SPHERE, 1, mat, r
        h[i].center[:] = list(c)
    for k, col in enumerate(_COLOURS):
        m[k].type = abi.RT_METAL if k == 7 else abi.RT_LAMBERTIAN
        m[k].fuzz = 0.0
        m[k].albedo.type, m[k].albedo.image = abi.RT_CONSTANT, -1
        m[k].albedo.color[:] = list(col)
    return scenes.Scene(h, m, [])


def adversarial_scene_large(extra: int = 12) -> scenes.Scene:
    """The adversarial scene plus `extra` small Lambertian spheres floating above it (17+ primitives: beyond the flat
    kernels' size limit, kept on them by the touching rectangles)."""
    base = adversarial_scene()
    n = len(base.hittables) + extra
    h = (abi.HittableDesc * n)()
    for i in range(len(base.hittables)):
        h[i] = base.hittables[i]
    for k in range(extra):
        i = len(base.hittables) + k
        h[i].type, h[i].is_active, h[i].material, h[i].radius = abi.RT_SPHERE, 1, k % 5, 0.15
        h[i].center[:] = [-1.8 + 0.35 * k, 1.6 + 0.1 * (k % 3), 0.8 + 0.2 * (k % 4)]
    return scenes.Scene(h, base.materials, [])


def adversarial_scene_tiled(n: int = 8) -> scenes.Scene:
    """The adversarial scene with its floor replaced by an n × n grid of abutting 1 × 1 floor tiles (XZRect, y = -1,
    shared edges on every side) and a second, overlapping copy of its middle row (exact ties in t over the overlap):
    8 + n·n + n primitives — beyond the flat kernels' 64 (kFlatMaxPrims), so only the BVH kernels render it, and its
    touching geometry is where the reference's culling parts from the geometric closest hit."""
    base = adversarial_scene()
    tiles = [(x, z) for z in range(n) for x in range(n)] + [(x, n // 2) for x in range(n)]
    nb = len(base.hittables)
    h = (abi.HittableDesc * (nb + len(tiles)))()
    for i in range(nb):
        h[i] = base.hittables[i]
    for k, (x, z) in enumerate(tiles):
        i = nb + k
        h[i].type, h[i].is_active, h[i].material = abi.RT_XZRECT, 1, (x + z + (k >= n * n)) % 5
        h[i].center[:] = [-n / 2 + 0.5 + x, -1.0, -n / 2 + 2.5 + z]
        h[i].width, h[i].height = 1.0, 1.0
    return scenes.Scene(h, base.materials, [])
