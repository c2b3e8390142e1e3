"""ctypes wrapper over oracle/build/liboracle.so -- TEST INFRASTRUCTURE ONLY.

The oracle is the CPU restatement of the reference ray tracer (see rt_oracle.h for the reference
file:line map). Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this.
"""
import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.environ.get("RT_ORACLE_LIB") or os.path.join(_HERE, "build", "liboracle.so")
_lib = None

F32P = np.ctypeslib.ndpointer(np.float32, flags="C_CONTIGUOUS")
I32P = np.ctypeslib.ndpointer(np.int32, flags="C_CONTIGUOUS")
U32P = np.ctypeslib.ndpointer(np.uint32, flags="C_CONTIGUOUS")

KAT_OPS = ["DOT", "NORMALIZED", "CROSS", "M3V3", "AFF_V3", "M4V4", "M3INV", "AFF_INV", "SHAPE",
           "OFFSET_001", "OFFSET_003", "REFLECT", "PHONG_R", "NRM_INTERP", "NORM", "CENTER", "SCREEN"]


class Camera(C.Structure):
    _fields_ = [("view", C.c_float * 16), ("viewport", C.c_float * 4), ("fovy", C.c_float),
                ("aspect", C.c_float)]


class RenderOpts(C.Structure):
    _fields_ = [("max_depth", C.c_int32), ("shadows", C.c_int32), ("background", C.c_float * 3),
                ("def_mat", C.c_float * 12), ("dir_lights6", C.c_void_p), ("n_dir_lights", C.c_int32),
                ("box_colors3", C.c_void_p)]


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            raise RuntimeError(f"oracle library missing: {_LIB_PATH} (run `make -C oracle`)")
        L = C.CDLL(_LIB_PATH)
        vp = C.c_void_p
        L.orc_mesh_load_obj.argtypes = [C.c_char_p, C.POINTER(vp)]
        L.orc_mesh_from_arrays.argtypes = [C.c_int32, F32P, vp, C.c_int32, I32P, U32P, I32P, C.c_int32,
                                           F32P, C.POINTER(vp)]
        L.orc_mesh_free.argtypes = [vp]
        L.orc_mesh_set_model.argtypes = [vp, F32P]
        L.orc_mesh_set_model.restype = None
        L.orc_mesh_counts.argtypes = [vp, C.POINTER(C.c_int32), C.POINTER(C.c_int32), C.POINTER(C.c_int32)]
        L.orc_mesh_export.argtypes = [vp] + [vp] * 8
        L.orc_generate_soup.argtypes = [C.c_int32, C.c_uint64, F32P]
        L.orc_scene_build.argtypes = [vp, C.c_int32, C.c_int32, C.POINTER(vp)]
        L.orc_scene_free.argtypes = [vp]
        L.orc_scene_box_count.argtypes = [vp]
        L.orc_scene_box_count.restype = C.c_int32
        L.orc_scene_boxes.argtypes = [vp, vp, vp, vp]
        L.orc_scene_pass_counts.argtypes = [vp, I32P, C.c_int32]
        L.orc_scene_pass_counts.restype = C.c_int32
        L.orc_camera_flycam.argtypes = [C.c_int32, C.c_int32, C.c_float, C.c_float, C.c_float, C.POINTER(Camera)]
        L.orc_camera_ray.argtypes = [C.POINTER(Camera), C.c_int32, C.c_int32, F32P, F32P]
        L.orc_render_opts_default.argtypes = [C.POINTER(RenderOpts), C.c_int32]
        L.orc_render.argtypes = [vp, C.POINTER(Camera), F32P, C.c_int32, C.c_int32, C.c_int32,
                                 C.POINTER(RenderOpts), C.c_int32, vp, C.c_int32, vp, vp, vp]
        L.orc_closest.argtypes = [vp, C.c_int32, F32P, F32P, I32P, F32P, F32P]
        L.orc_shadow.argtypes = [vp, C.c_int32, F32P, F32P, I32P]
        L.orc_kat.argtypes = [C.c_int32, C.c_int32, F32P, F32P]
        L.orc_box_colors_glibc.argtypes = [C.c_int32, F32P]
        L.orc_last_error.restype = C.c_char_p
        _lib = L
    return _lib


def _p(a):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


def _check(rc):
    if rc != 0:
        raise RuntimeError("oracle: " + lib().orc_last_error().decode())


class Mesh:
    """Tucano-semantics mesh (objimporter.hpp / mesh.hpp) held by the oracle."""

    def __init__(self, handle):
        self.h = handle

    @classmethod
    def load_obj(cls, path):
        h = C.c_void_p()
        _check(lib().orc_mesh_load_obj(os.fsencode(path), C.byref(h)))
        return cls(h)

    @classmethod
    def from_arrays(cls, v3, faces, materials, vn3=None, groups=None):
        """v3 [nv,3] f32; faces [nf,3] u32; materials [nm,12]; groups: list of (n_faces, mat_id)."""
        v3 = np.ascontiguousarray(v3, np.float32)
        faces = np.ascontiguousarray(faces, np.uint32).reshape(-1)
        mats = np.ascontiguousarray(materials, np.float32).reshape(-1, 12)
        if groups is None:
            groups = [(len(faces) // 3, 0 if len(mats) else -1)]
        gc = np.array([3 * g[0] for g in groups], np.int32)
        gm = np.array([g[1] for g in groups], np.int32)
        vn = None if vn3 is None else np.ascontiguousarray(vn3, np.float32)
        h = C.c_void_p()
        _check(lib().orc_mesh_from_arrays(len(v3), v3, _p(vn), len(gc), gc, faces, gm, len(mats),
                                          mats.reshape(-1) if len(mats) else np.zeros(12, np.float32),
                                          C.byref(h)))
        return cls(h)

    def set_model(self, model16):
        """Model::modelMatrix (column-major 4x4 affine): getShapeModelMatrix() = model16 * normalisation."""
        lib().orc_mesh_set_model(self.h, np.ascontiguousarray(model16, np.float32).reshape(16))

    def counts(self):
        a, b, c = C.c_int32(), C.c_int32(), C.c_int32()
        lib().orc_mesh_counts(self.h, C.byref(a), C.byref(b), C.byref(c))
        return a.value, b.value, c.value

    def export(self):
        nv, nf, nm = self.counts()
        d = dict(v4=np.zeros((nv, 4), np.float32), vn3=np.zeros((nv, 3), np.float32),
                 fidx=np.zeros((nf, 3), np.uint32), fn3=np.zeros((nf, 3), np.float32),
                 fmat=np.zeros(nf, np.int32), mats=np.zeros((max(nm, 1), 12), np.float32),
                 M16=np.zeros(16, np.float32), sc4=np.zeros(4, np.float32))
        lib().orc_mesh_export(self.h, *[_p(d[k]) for k in ("v4", "vn3", "fidx", "fn3", "fmat", "mats", "M16", "sc4")])
        d["mats"] = d["mats"][:nm]
        return d

    def __del__(self):
        if getattr(self, "h", None) and _lib is not None:
            _lib.orc_mesh_free(self.h)
            self.h = None


def generate_soup(n_tris, seed=12345):
    v = np.zeros((3 * n_tris, 3), np.float32)
    lib().orc_generate_soup(n_tris, seed, v)
    return v


class Scene:
    def __init__(self, mesh, min_faces=300, max_boxes=2**31 - 1):
        self.mesh = mesh
        self.h = C.c_void_p()
        _check(lib().orc_scene_build(mesh.h, min_faces, max_boxes, C.byref(self.h)))

    def box_count(self):
        return lib().orc_scene_box_count(self.h)

    def boxes(self):
        nb = self.box_count()
        nf = self.mesh.counts()[1]
        b6 = np.zeros((nb, 6), np.float32)
        cnt = np.zeros(nb, np.int32)
        order = np.zeros(nf, np.int32)
        lib().orc_scene_boxes(self.h, _p(b6), _p(cnt), _p(order))
        return b6, cnt, order

    def pass_counts(self):
        out = np.zeros(4096, np.int32)
        n = lib().orc_scene_pass_counts(self.h, out, 4096)
        return out[:n].tolist()

    def closest(self, o, d):
        o = np.ascontiguousarray(o, np.float32).reshape(-1, 3)
        d = np.ascontiguousarray(d, np.float32).reshape(-1, 3)
        n = len(o)
        face = np.zeros(n, np.int32)
        t = np.zeros(n, np.float32)
        P = np.zeros((n, 3), np.float32)
        lib().orc_closest(self.h, n, o, d, face, t, P)
        return face, t, P

    def shadow(self, P, L):
        P = np.ascontiguousarray(P, np.float32).reshape(-1, 3)
        L = np.ascontiguousarray(L, np.float32).reshape(-1, 3)
        out = np.zeros(len(P), np.int32)
        lib().orc_shadow(self.h, len(P), P, L, out)
        return out

    def render(self, cam, lights, W, H, full=False, pixels=None, threads=1, dir_lights=(), max_depth=None,
               box_colors=None):
        """lights: [(pos3, color3), ...] point lights; dir_lights: [(vector3, color3), ...] directional lights
        (Flyscene::dirLights). max_depth overrides traceRay's recursion limit (flyscene.hpp:142; FULL = 2
        with shadows, PRIMARY = 1 without). box_colors [nb,3]: RENDER_BOUNDINGBOX_COLORED_TRIANGLES
        (flyscene.cpp:334-348). Returns rgb [n,3], face [n], t [n] (n = W*H or len(pixels))."""
        opts = RenderOpts()
        lib().orc_render_opts_default(C.byref(opts), 1 if full else 0)
        if max_depth is not None:
            opts.max_depth = max_depth
        if box_colors is not None:
            BC = np.ascontiguousarray(box_colors, np.float32).reshape(-1)
            assert BC.size == 3 * self.box_count()
            opts.box_colors3 = BC.ctypes.data
        D6 = np.ascontiguousarray(np.array([list(p) + list(c) for p, c in dir_lights], np.float32).reshape(-1))
        opts.dir_lights6 = D6.ctypes.data if len(dir_lights) else None
        opts.n_dir_lights = len(dir_lights)
        L6 = np.ascontiguousarray(np.array([list(p) + list(c) for p, c in lights], np.float32).reshape(-1))
        if pixels is None:
            n = W * H
            pix = None
        else:
            pix = np.ascontiguousarray(pixels, np.int32).reshape(-1, 2)
            n = len(pix)
        rgb = np.zeros((n, 3), np.float32)
        face = np.zeros(n, np.int32)
        t = np.zeros(n, np.float32)
        _check(lib().orc_render(self.h, C.byref(cam), L6, len(lights), W, H, C.byref(opts), n, _p(pix),
                                threads, _p(rgb), _p(face), _p(t)))
        return rgb, face, t

    def __del__(self):
        if getattr(self, "h", None) and _lib is not None:
            _lib.orc_scene_free(self.h)
            self.h = None


def flycam(W, H, dx=0.0, dy=0.0, dz=0.0):
    c = Camera()
    lib().orc_camera_flycam(W, H, dx, dy, dz, C.byref(c))
    return c


def camera_ray(cam, i, j):
    o = np.zeros(3, np.float32)
    d = np.zeros(3, np.float32)
    lib().orc_camera_ray(C.byref(cam), i, j, o, d)
    return o, d


def box_colors_glibc(n):
    """BoundingBox::setRandomColor for n boxes of a fresh reference process (glibc srand(1) + rand())."""
    out = np.zeros((n, 3), np.float32)
    lib().orc_box_colors_glibc(n, out)
    return out


def kat(op, inp, n, out_len):
    out = np.zeros(n * out_len, np.float32)
    _check(lib().orc_kat(op, n, np.ascontiguousarray(inp, np.float32), out))
    return out


DEFAULT_LIGHTS = [((-0.5, 2.0, 3.0), (1.0, 1.0, 1.0))]  # flyscene.cpp:37
