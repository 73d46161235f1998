"""Builds the reference's scene pointer graph (include/rt_reference_graph.h layouts) in host memory.

This is what the reference viewer hands to LaunchKernel as `Hittable* world`: CudaLayer::GenerateWorld's
Hittable → ObjectUnion → Sphere/Rect → Material → ObjectUnion → Lambertian/... → Texture → ... chain
(CudaLayer.cpp:131-245) under a BVHNode tree built as the BVHNode constructor does (Hittable.cuh:303-385:
drop inactive, stable sort by type, split at the first type boundary or at the middle in list order).
"""
from __future__ import annotations

import ctypes as C

from cudaraytracer_amd import abi

RTREF_BVHNODE = 5


class Vec3(C.Structure):
    _fields_ = [("e", C.c_float * 3)]


class Hittable(C.Structure):
    _fields_ = [("type", C.c_int32), ("is_active", C.c_uint8), ("pad_", C.c_uint8 * 3), ("object", C.c_void_p)]


class Sphere(C.Structure):
    _fields_ = [("center", Vec3), ("radius", C.c_float), ("mat_ptr", C.c_void_p)]


class Rect(C.Structure):
    _fields_ = [("center", Vec3), ("width", C.c_float), ("height", C.c_float), ("mat_ptr", C.c_void_p)]


class AABB(C.Structure):
    _fields_ = [("minimum", Vec3), ("maximum", Vec3)]


class BVHNode(C.Structure):
    _fields_ = [("box", AABB), ("left", C.c_void_p), ("right", C.c_void_p), ("memory", C.c_void_p)]


class Material(C.Structure):
    _fields_ = [("type", C.c_int32), ("object", C.c_void_p)]


class Lambertian(C.Structure):
    _fields_ = [("albedo", C.c_void_p)]


class Metal(C.Structure):
    _fields_ = [("albedo", C.c_void_p), ("fuzz", C.c_float)]


class Dielectric(C.Structure):
    _fields_ = [("ir", C.c_float)]


class DiffuseLight(C.Structure):
    _fields_ = [("albedo", C.c_void_p), ("light_intensity", C.c_int32)]


class Texture(C.Structure):
    _fields_ = [("type", C.c_int32), ("object", C.c_void_p)]


class Constant(C.Structure):
    _fields_ = [("color", Vec3), ("padding", C.c_float)]


class Checker(C.Structure):
    _fields_ = [("odd", C.c_void_p), ("even", C.c_void_p)]


class Image(C.Structure):
    _fields_ = [("data", C.c_void_p), ("path", C.c_char_p), ("width", C.c_int32), ("height", C.c_int32),
                ("bytes_per_scanline", C.c_int32)]


assert C.sizeof(Hittable) == 16 and C.sizeof(Sphere) == 24 and C.sizeof(Rect) == 32
assert C.sizeof(BVHNode) == 48 and C.sizeof(Material) == 16 and C.sizeof(Texture) == 16
assert C.sizeof(Constant) == 16 and C.sizeof(Metal) == 16 and C.sizeof(Image) == 32


class Graph:
    """Owns every ctypes object of the graph (keeps the memory alive)."""

    def __init__(self):
        self.keep = []
        self.world = None

    def _new(self, obj):
        self.keep.append(obj)
        return obj

    def _union(self, target) -> int:
        u = self._new(C.c_void_p(C.addressof(target)))  # ObjectUnion: one pointer
        return C.addressof(u)

    def texture(self, t: abi.TextureDesc, images) -> int:
        tex = self._new(Texture())
        tex.type = t.type
        if t.type == abi.RT_CONSTANT:
            obj = self._new(Constant(Vec3((C.c_float * 3)(*t.color))))
        elif t.type == abi.RT_CHECKER:
            odd = self._new(Constant(Vec3((C.c_float * 3)(*t.color))))
            even = self._new(Constant(Vec3((C.c_float * 3)(*t.color2))))
            obj = self._new(Checker(C.addressof(odd), C.addressof(even)))
        else:
            im = images[t.image] if 0 <= t.image < len(images) else None
            obj = self._new(Image())
            if im is not None:
                obj.data = im.ctypes.data
                obj.height, obj.width = int(im.shape[0]), int(im.shape[1])
                obj.bytes_per_scanline = 3 * obj.width
        tex.object = self._union(obj)
        return C.addressof(tex)

    def material(self, m: abi.MaterialDesc, images) -> int:
        mat = self._new(Material())
        mat.type = m.type
        if m.type == abi.RT_LAMBERTIAN:
            obj = self._new(Lambertian(self.texture(m.albedo, images)))
        elif m.type == abi.RT_METAL:
            obj = self._new(Metal(self.texture(m.albedo, images), m.fuzz))
        elif m.type == abi.RT_DIELECTRIC:
            obj = self._new(Dielectric(m.ir))
        else:
            obj = self._new(DiffuseLight(self.texture(m.albedo, images), m.light_intensity))
        mat.object = self._union(obj)
        return C.addressof(mat)

    def hittable(self, h: abi.HittableDesc, m: abi.MaterialDesc, images) -> Hittable:
        hit = self._new(Hittable())
        hit.type = h.type
        hit.is_active = 1 if h.is_active else 0
        mp = self.material(m, images)
        if h.type == abi.RT_SPHERE:
            obj = self._new(Sphere(Vec3((C.c_float * 3)(*h.center)), h.radius, mp))
        else:
            obj = self._new(Rect(Vec3((C.c_float * 3)(*h.center)), h.width, h.height, mp))
        hit.object = self._union(obj)
        return hit

    @staticmethod
    def _box(h: Hittable) -> tuple:
        if h.type == RTREF_BVHNODE:
            node = BVHNode.from_address(C.c_void_p.from_address(h.object).value)
            return tuple(node.box.minimum.e), tuple(node.box.maximum.e)
        addr = C.c_void_p.from_address(h.object).value
        if h.type == abi.RT_SPHERE:
            s = Sphere.from_address(addr)
            c, r = s.center.e, s.radius
            return tuple(C.c_float(c[i] - r).value for i in range(3)), tuple(C.c_float(c[i] + r).value for i in range(3))
        r = Rect.from_address(addr)
        c = r.center.e
        w2, h2 = C.c_float(r.width / 2).value, C.c_float(r.height / 2).value
        lo, hi = [0.0] * 3, [0.0] * 3
        axes = {abi.RT_XYRECT: (0, 1, 2), abi.RT_XZRECT: (0, 2, 1), abi.RT_YZRECT: (2, 1, 0)}[h.type]
        # (width axis, height axis, plane axis)
        wa, ha, ka = axes
        lo[wa], hi[wa] = C.c_float(c[wa] - w2).value, C.c_float(c[wa] + w2).value
        lo[ha], hi[ha] = C.c_float(c[ha] - h2).value, C.c_float(c[ha] + h2).value
        lo[ka], hi[ka] = C.c_float(c[ka] - 0.0001).value, C.c_float(c[ka] + 0.0001).value
        return tuple(lo), tuple(hi)

    def bvh(self, objs: list) -> Hittable:
        """A BVHNODE hittable over `objs` (Hittable.cuh:303-385)."""
        node = self._new(BVHNode())
        active = [o for o in objs if o.is_active]
        if active:
            active = sorted(active, key=lambda o: o.type)  # stable
            if len(active) == 1:
                left = right = active[0]
            elif len(active) == 2:
                left, right = active
            else:
                mid = 0
                while mid < len(active) and active[mid].type == active[0].type:
                    mid += 1
                if mid == 0 or mid == len(active):
                    mid = len(active) // 2
                left, right = self.bvh(active[:mid]), self.bvh(active[mid:])
            node.left, node.right = C.addressof(left), C.addressof(right)
            (l0, l1), (r0, r1) = self._box(left), self._box(right)
            node.box.minimum.e[:] = [min(a, b) for a, b in zip(l0, r0)]
            node.box.maximum.e[:] = [max(a, b) for a, b in zip(l1, r1)]
        h = self._new(Hittable())
        h.type = RTREF_BVHNODE
        h.is_active = 1
        h.object = self._union(node)
        return h


def build_graph(scene) -> Graph:
    """Reference pointer graph of a cudaraytracer_amd.scenes.Scene (one material per hittable)."""
    g = Graph()
    objs = [g.hittable(scene.hittables[i], scene.materials[scene.hittables[i].material], scene.images)
            for i in range(scene.num_hittables)]
    g.world = g.bvh(objs)
    return g
