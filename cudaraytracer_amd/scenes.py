"""Scene descriptions and the BASELINE.json configurations (host side, no GPU needed).

`Scene` holds the flat description (rt_scene_desc) the C ABI takes: hittables in list order, one material
per hittable (as CudaLayer::GenerateWorld allocates them, CudaLayer.cpp:103-256) and optional RGB8 images.
The built-in generators live in librt_hip.so (csrc/builtin_scenes.cpp); the camera → InputStruct fill
follows CudaLayer.cpp:43-65.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field

import numpy as np

from . import abi
from ._lib import check, lib

SCENE_DEFAULT_WORLD = 0
SCENE_THREE_SPHERES = 1
SCENE_RTIOW = 2
SCENE_CORNELL = 3
SCENE_TEXTURED = 4

DEFAULT_BG_START = (1.0, 1.0, 1.0)  # CudaLayer.h:143
DEFAULT_BG_END = (0.5, 0.7, 1.0)  # CudaLayer.h:144


@dataclass
class Scene:
    hittables: C.Array
    materials: C.Array
    images: list = field(default_factory=list)  # numpy uint8 (H, W, 3) arrays, kept alive here
    _image_descs: C.Array | None = None

    @property
    def num_hittables(self) -> int:
        return len(self.hittables)

    def desc(self) -> abi.SceneDesc:
        imgs = (abi.ImageDesc * max(1, len(self.images)))()
        for i, im in enumerate(self.images):
            im = np.ascontiguousarray(im, dtype=np.uint8)
            self.images[i] = im
            imgs[i].data = im.ctypes.data
            imgs[i].height, imgs[i].width = int(im.shape[0]), int(im.shape[1])
        self._image_descs = imgs
        return abi.SceneDesc(
            C.cast(self.hittables, C.POINTER(abi.HittableDesc)),
            len(self.hittables),
            C.cast(self.materials, C.POINTER(abi.MaterialDesc)),
            len(self.materials),
            C.cast(imgs, C.POINTER(abi.ImageDesc)),
            len(self.images),
        )

    def hittables_bytes(self) -> bytes:
        return bytes(memoryview(self.hittables).cast("B"))

    def materials_bytes(self) -> bytes:
        return bytes(memoryview(self.materials).cast("B"))

    @classmethod
    def from_bytes(cls, hittables: bytes, materials: bytes, images=None) -> "Scene":
        nh = len(hittables) // C.sizeof(abi.HittableDesc)
        nm = len(materials) // C.sizeof(abi.MaterialDesc)
        h = (abi.HittableDesc * nh).from_buffer_copy(hittables)
        m = (abi.MaterialDesc * nm).from_buffer_copy(materials)
        return cls(h, m, list(images or []))


TEXTURE_EARTH, TEXTURE_MOON, TEXTURE_SUN = 0, 1, 2
DEFAULT_TEXTURE_SIZE = (1024, 512)  # parity fixtures; BASELINE config 5 uses the reference's 8192x4096


def procedural_texture(kind: int = TEXTURE_EARTH, width: int = 1024, height: int = 512) -> np.ndarray:
    """Deterministic RGB8 (H, W, 3) stand-in for the reference's 8K planet maps (assets/textures/8k_*.jpg;
    there is no JPEG decoder here): rt_procedural_texture in librt_hip.so (host code, no device needed)."""
    img = np.empty((height, width, 3), dtype=np.uint8)
    check(lib().rt_procedural_texture(kind, width, height, img.ctypes.data), "rt_procedural_texture")
    return img


def load_image(filename: str) -> np.ndarray | None:
    """The reference's LoadImage (Utils/RawStbImage.h:11-22, stbi_load with desired_channels 0): the decoded file as
    (height, width, channels) uint8, row 0 at the top, channels as stored (3 for the reference's 8K planet maps, which
    is what Image::value reads, Texture.cuh:76), or None when the file cannot be decoded — the reference logs the
    error and hands back a null pointer (CudaLayer.cpp:895).  Decoding is host work and uses Pillow; Pillow's
    libjpeg and stb's decoder may round some texels differently (parity unpinned against stb)."""
    try:
        from PIL import Image as _PIL
    except ImportError as e:  # pragma: no cover - Pillow is part of this image
        raise RuntimeError("load_image needs Pillow to decode image files") from e
    try:
        with _PIL.open(filename) as im:
            im.load()
            if im.mode not in ("L", "LA", "RGB", "RGBA"):
                im = im.convert("RGBA" if "A" in im.getbands() else "RGB")
            a = np.asarray(im, dtype=np.uint8)
    except (OSError, ValueError):
        return None
    return np.ascontiguousarray(a if a.ndim == 3 else a[:, :, None])


def builtin(which: int, seed: int = 1, texture_size: tuple = DEFAULT_TEXTURE_SIZE, images: list | None = None) -> Scene:
    """Built-in scene `which` (see rt_builtin_scene in include/rt_hip.h).  The textured scene gets three
    procedural images (earth, moon, sun) of texture_size = (width, height), or the caller's `images` — RGB8
    (H, W, 3) arrays, e.g. from load_image on the reference's assets/textures files."""
    L = lib()
    nh, nm = C.c_uint32(0), C.c_uint32(0)
    check(L.rt_builtin_scene(which, seed, None, C.byref(nh), None, C.byref(nm)), "rt_builtin_scene(size)")
    h = (abi.HittableDesc * nh.value)()
    m = (abi.MaterialDesc * nm.value)()
    check(L.rt_builtin_scene(which, seed, h, C.byref(nh), m, C.byref(nm)), "rt_builtin_scene")
    imgs = []
    if which == SCENE_TEXTURED and images is not None:
        if len(images) != 3 or any(im.ndim != 3 or im.shape[2] != 3 or im.dtype != np.uint8 for im in images):
            raise ValueError("the textured scene takes three RGB8 (H, W, 3) uint8 images (earth, moon, sun)")
        imgs = [np.ascontiguousarray(im) for im in images]
    elif which == SCENE_TEXTURED:
        w, hh = texture_size
        imgs = [procedural_texture(k, w, hh) for k in (TEXTURE_EARTH, TEXTURE_MOON, TEXTURE_SUN)]
    return Scene(h, m, imgs)


def camera_inputs(position, orientation, fov_degrees, near=0.1, far=10.0, world_up=(0.0, 1.0, 0.0),
                  bg_start=DEFAULT_BG_START, bg_end=DEFAULT_BG_END) -> abi.InputStruct:
    """InputStruct from a Camera (Renderer/Camera.h:39-45) exactly as CudaLayer.cpp:43-65 fills it."""
    F3 = C.c_float * 3
    out = abi.InputStruct()
    lib().rt_camera_inputs(F3(*position), F3(*orientation), F3(*world_up), fov_degrees, near, far,
                           F3(*bg_start), F3(*bg_end), C.byref(out))
    return out


def normalized(v) -> tuple:
    a = np.asarray(v, dtype=np.float32)
    inv = np.float32(1.0) / np.sqrt(np.float32(a @ a), dtype=np.float32)
    return tuple(float(x) for x in (a * inv).astype(np.float32))


@dataclass
class Config:
    name: str
    scene: int
    width: int
    height: int
    spp: int
    depth: int
    position: tuple
    orientation: tuple
    fov: float
    bg_start: tuple = DEFAULT_BG_START
    bg_end: tuple = DEFAULT_BG_END
    description: str = ""
    texture_size: tuple = DEFAULT_TEXTURE_SIZE  # (width, height) of the textured scene's images

    def inputs(self) -> abi.InputStruct:
        return camera_inputs(self.position, self.orientation, self.fov, bg_start=self.bg_start, bg_end=self.bg_end)

    def scene_desc(self) -> Scene:
        """The configuration's scene, with its textures at the configured size."""
        return builtin(self.scene, texture_size=self.texture_size)

    def scaled(self, width: int, height: int, spp: int | None = None) -> "Config":
        c = Config(**{k: getattr(self, k) for k in self.__dataclass_fields__})
        c.width, c.height = width, height
        if spp is not None:
            c.spp = spp
        return c


_RTIOW_FWD = normalized((-13.0, -2.0, -3.0))
_TEX_FWD = normalized((0.0, -0.2, -1.0))

# BASELINE.json "configs" 
CONFIGS = {
    "c1": Config("c1", SCENE_THREE_SPHERES, 400, 225, 4, 4, (0.0, 0.0, 1.0), (0.0, 0.0, -1.0), 45.0,
                 description="400x225, 4 spp, depth 4, 3-sphere Lambertian scene (CPU reference path)"),
    "c2": Config("c2", SCENE_RTIOW, 1920, 1080, 64, 8, (13.0, 2.0, 3.0), _RTIOW_FWD, 20.0,
                 description="1920x1080, 64 spp, depth 8, RTIOW final random-spheres scene"),
    "c3": Config("c3", SCENE_CORNELL, 3840, 2160, 256, 16, (278.0, 278.0, -800.0), (0.0, 0.0, 1.0), 40.0,
                 bg_start=(0.0, 0.0, 0.0), bg_end=(0.0, 0.0, 0.0),
                 description="3840x2160, 256 spp, depth 16, Cornell-box-style emissive scene"),
    "c4": Config("c4", SCENE_RTIOW, 7680, 4320, 128, 8, (13.0, 2.0, 3.0), _RTIOW_FWD, 20.0,
                 description="8 GPUs, 7680x4320, 128 spp, depth 8, RTIOW (image-tile split + gather)"),
    "c5": Config("c5", SCENE_TEXTURED, 1920, 1080, 1, 4, (0.0, 2.0, 10.0), _TEX_FWD, 45.0,
                 description="1920x1080, 1 spp progressive, depth 4, textured spheres + moving camera",
                 texture_size=(8192, 4096)),
    "default": Config("default", SCENE_DEFAULT_WORLD, 800, 600, 36, 12, (0.0, 2.0, 12.0), (0.0, 0.0, -1.0), 45.0,
                      description="the reference viewer's startup state (CudaLayer.h:66-67, 123-124)"),
}


def sphere_field(n: int, seed: int) -> Scene:
    """n small random spheres (Lambertian / metal / dielectric) over RTIOW's ground, under config 2's camera: the
    large scenes the reference viewer grows with AddHittable (CudaLayer.cpp:918-1370)."""
    rng = np.random.default_rng(seed)
    h = (abi.HittableDesc * (n + 1))()
    m = (abi.MaterialDesc * 4)()
    for k, (t, f) in enumerate([(abi.RT_LAMBERTIAN, 0.0), (abi.RT_METAL, 0.3), (abi.RT_DIELECTRIC, 0.0),
                                (abi.RT_LAMBERTIAN, 0.0)]):
        m[k].type, m[k].fuzz, m[k].ir = t, f, 1.5
        m[k].albedo.type, m[k].albedo.image = abi.RT_CONSTANT, -1
        m[k].albedo.color[:] = [0.5, 0.6 - 0.1 * k, 0.3 + 0.1 * k]
    h[0].type, h[0].is_active, h[0].material, h[0].radius = abi.RT_SPHERE, 1, 3, 1000.0
    h[0].center[:] = [0.0, -1000.0, 0.0]
    xyz = rng.uniform([-11.0, 0.05, -11.0], [11.0, 2.5, 11.0], (n, 3)).astype(np.float32)
    rad = rng.uniform(0.03, 0.15, n).astype(np.float32)
    mat = rng.integers(0, 3, n)
    for i in range(n):
        h[i + 1].type, h[i + 1].is_active = abi.RT_SPHERE, 1
        h[i + 1].center[:] = [float(v) for v in xyz[i]]
        h[i + 1].radius, h[i + 1].material = float(rad[i]), int(mat[i])
    return Scene(h, m, [])


def moving_camera(frame: int, frames: int = 60) -> tuple:
    """C5's scripted camera path: an orbit around the scene (position, orientation)."""
    ang = 2.0 * np.pi * frame / max(1, frames)
    pos = (float(10.0 * np.sin(ang)), 2.0, float(10.0 * np.cos(ang)))
    fwd = normalized((-pos[0], -1.5, -pos[2]))
    return pos, fwd
