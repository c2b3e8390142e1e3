"""ctypes binding of librtamd.so (include/rt/rt_api.h) for tests and bench.py.

Plumbing only: the product is the C ABI + gfx950 kernels. Loading fails loudly if the built library
is missing (there is no Python or CPU fallback for any render/trace call).
"""
import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# RTAMD_LIB: an A/B build of the same library (`make ablib`), for measurements only
LIB_PATH = os.environ.get("RTAMD_LIB") or os.path.join(HERE, "lib", "librtamd.so")

RT_MODE_PRIMARY = 0
RT_MODE_FULL = 1
RT_MODE_BOX_COLORS = 2  # RENDER_BOUNDINGBOX_COLORED_TRIANGLES (flyscene.hpp:166, flyscene.cpp:334-348)
RT_FRAME_WRITE_HITS = 1
RT_FRAME_STATS = 2
RT_FRAME_TIMELINE = 4
RT_FRAME_WAVE_STATS = 8
RT_DEVICE_NONE = -2

# Every symbol include/rt/rt_api.h declares (checked by tests/test_abi.py)
EXPORTS = [
    "rt_mesh_load_obj", "rt_mesh_from_arrays", "rt_mesh_destroy", "rt_mesh_get_desc", "rt_generate_soup",
    "rt_write_ppm", "rt_scene_opts_default", "rt_scene_create", "rt_scene_destroy", "rt_scene_get_info",
    "rt_scene_ref_boxes", "rt_camera_flycam", "rt_render", "rt_render_async", "rt_synchronize",
    "rt_frame_download", "rt_trace_closest", "rt_trace_shadow", "rt_device_count", "rt_version",
    "rt_last_error", "rt_debug_math_host", "rt_debug_math_device", "rt_debug_validate_bvh",
    "rt_debug_set_variant", "rt_scene_save", "rt_scene_load",
    "rt_frame_download_rgb8", "rt_write_ppm_rgb8", "rt_frame_shard_bytes", "rt_frame_pack_shard_rgb8",
    "rt_frame_unpack_shards_rgb8", "rt_rand_seed", "rt_rand", "rt_lights_spherical", "rt_light_directional",
    "rt_trace_closest_normal", "rt_trace_color", "rt_debug_ray", "rt_version_string", "rt_source_hash",
    "rt_debug_timeline", "rt_debug_counters", "rt_box_colors_random", "rt_scene_set_box_colors", "rt_frame_shard_tiles",
    "rt_debug_record_layout", "rt_debug_scene_flags", "rt_debug_env_knobs", "rt_debug_tree_cost",
    "rt_synchronize_devices", "rt_debug_lpt_stats", "rt_debug_wave_stats",
]
RT_MAX_DEVICES = 16
RT_DEVICES_ALL = -1


class Material(C.Structure):
    _fields_ = [("ka", C.c_float * 3), ("kd", C.c_float * 3), ("ks", C.c_float * 3), ("shininess", C.c_float),
                ("optical_density", C.c_float), ("dissolve", C.c_float)]


class MeshDesc(C.Structure):
    _fields_ = [("n_vertices", C.c_int32), ("vertices", C.c_void_p), ("vertex_normals", C.c_void_p),
                ("n_faces", C.c_int32), ("face_vertex_ids", C.c_void_p), ("face_normals", C.c_void_p),
                ("face_material_ids", C.c_void_p), ("n_materials", C.c_int32), ("materials", C.c_void_p),
                ("shape_model_matrix", C.c_float * 16)]


class SceneOpts(C.Structure):
    _fields_ = [("device", C.c_int32), ("min_faces", C.c_int32), ("max_boxes", C.c_int32),
                ("leaf_size", C.c_int32), ("default_material", Material), ("background", C.c_float * 3),
                ("frames_in_flight", C.c_int32), ("builder", C.c_int32), ("box_builder", C.c_int32),
                ("wide_tree", C.c_int32), ("n_devices", C.c_int32), ("devices", C.c_int32 * 16)]


class SceneInfo(C.Structure):
    _fields_ = [("n_faces", C.c_int32), ("n_vertices", C.c_int32), ("n_ref_boxes", C.c_int32),
                ("bvh_nodes", C.c_int32), ("bvh_leaves", C.c_int32), ("bvh_depth", C.c_int32),
                ("device_bytes", C.c_int64), ("build_ms", C.c_double), ("device", C.c_int32),
                ("prep_ms", C.c_double), ("boxes_ms", C.c_double), ("bvh_ms", C.c_double), ("upload_ms", C.c_double),
                ("builder", C.c_int32), ("bvh_gpu_ms", C.c_double), ("box_builder", C.c_int32),
                ("boxes_gpu_ms", C.c_double), ("wide_nodes", C.c_int32), ("wide_depth", C.c_int32),
                ("n_devices", C.c_int32), ("replicate_ms", C.c_double)]


class Camera(C.Structure):
    _fields_ = [("view_matrix", C.c_float * 16), ("viewport", C.c_float * 4), ("fovy", C.c_float),
                ("aspect_ratio", C.c_float)]


class RaySegment(C.Structure):
    _fields_ = [("origin", C.c_float * 3), ("direction", C.c_float * 3), ("length", C.c_float),
                ("color", C.c_float * 3)]


class Light(C.Structure):
    _fields_ = [("position", C.c_float * 3), ("color", C.c_float * 3), ("kind", C.c_int32)]


RT_LIGHT_POINT, RT_LIGHT_DIRECTIONAL = 0, 1


class RandState(C.Structure):
    _fields_ = [("r", C.c_uint32 * 34), ("k", C.c_uint32)]


class Frame(C.Structure):
    _fields_ = [("width", C.c_int32), ("height", C.c_int32), ("mode", C.c_int32), ("shard_index", C.c_int32),
                ("shard_count", C.c_int32), ("flags", C.c_int32), ("max_depth", C.c_int32)]


class Stats(C.Structure):
    _fields_ = [("kernel_ms", C.c_double), ("launches", C.c_int64), ("trace_kernel_ms", C.c_double),
                ("primary_rays", C.c_int64), ("total_rays", C.c_int64),
                ("hits", C.c_int64), ("node_visits", C.c_int64), ("tri_tests", C.c_int64),
                ("wave_node_fetches", C.c_int64), ("wave_tri_fetches", C.c_int64), ("wave_node_bytes", C.c_int64)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"librtamd.so not built: {LIB_PATH} (run `make` or __graft_entry__.build())")
        L = C.CDLL(LIB_PATH)
        vp = C.c_void_p
        L.rt_last_error.restype = C.c_char_p
        L.rt_version_string.restype = C.c_char_p
        L.rt_source_hash.restype = C.c_char_p
        L.rt_mesh_load_obj.argtypes = [C.c_char_p, C.POINTER(vp)]
        L.rt_mesh_from_arrays.argtypes = [C.c_int32, vp, vp, C.c_int32, vp, vp, vp, C.c_int32, vp, C.POINTER(vp)]
        L.rt_mesh_destroy.argtypes = [vp]
        L.rt_mesh_get_desc.argtypes = [vp, C.POINTER(MeshDesc)]
        L.rt_generate_soup.argtypes = [C.c_int32, C.c_uint64, vp]
        L.rt_generate_soup.restype = None
        L.rt_write_ppm.argtypes = [C.c_char_p, vp, C.c_int32, C.c_int32]
        L.rt_scene_opts_default.argtypes = [C.POINTER(SceneOpts)]
        L.rt_scene_opts_default.restype = None
        L.rt_scene_create.argtypes = [C.POINTER(MeshDesc), C.POINTER(SceneOpts), C.POINTER(vp)]
        L.rt_scene_destroy.argtypes = [vp]
        L.rt_scene_destroy.restype = None
        L.rt_scene_get_info.argtypes = [vp, C.POINTER(SceneInfo)]
        L.rt_scene_ref_boxes.argtypes = [vp, vp, vp, vp]
        L.rt_camera_flycam.argtypes = [C.c_int32, C.c_int32, C.c_float, C.c_float, C.c_float, C.POINTER(Camera)]
        L.rt_camera_flycam.restype = None
        L.rt_render.argtypes = [vp, C.POINTER(Camera), vp, C.c_int32, C.POINTER(Frame), vp, C.POINTER(Stats)]
        L.rt_render_async.argtypes = [vp, C.POINTER(Camera), vp, C.c_int32, C.POINTER(Frame)]
        L.rt_synchronize.argtypes = [vp, C.POINTER(Stats)]
        L.rt_synchronize_devices.argtypes = [vp, C.POINTER(Stats), C.c_int32, vp]
        L.rt_frame_download.argtypes = [vp, C.c_int64, vp, vp, vp]
        L.rt_trace_closest.argtypes = [vp, C.c_int32, vp, vp, vp, vp, vp]
        L.rt_trace_shadow.argtypes = [vp, C.c_int32, vp, vp, vp]
        L.rt_debug_math_host.argtypes = [C.c_int32, C.c_int32, vp, vp]
        L.rt_debug_math_device.argtypes = [C.c_int32, C.c_int32, vp, vp]
        L.rt_debug_validate_bvh.argtypes = [vp, vp]
        L.rt_debug_record_layout.argtypes = [C.c_int64, C.c_int64, C.c_int64, vp]
        L.rt_debug_scene_flags.argtypes = [vp, vp, vp, vp]
        L.rt_debug_tree_cost.argtypes = [vp, C.c_double, vp]
        L.rt_debug_set_variant.argtypes = [C.c_int32]
        L.rt_debug_env_knobs.argtypes = [C.c_int32]
        # A/B and diagnostic environment knobs (RT_KERNEL_VARIANT, RT_SPLIT_K, RT_SAH_TRAV, RT_TIMING, ...):
        # the library ignores the environment unless asked; measurement scripts opt in explicitly
        if os.environ.get("RTAMD_DEBUG_KNOBS") == "1":
            L.rt_debug_env_knobs(1)
        L.rt_debug_timeline.argtypes = [vp, C.c_int64, vp, C.POINTER(C.c_int64)]
        L.rt_debug_counters.argtypes = [vp, C.c_int64, C.POINTER(C.c_int64)]
        # (earlier API 4 builds, loaded for A/B through RTAMD_LIB, lack these)
        if hasattr(L, "rt_debug_lpt_stats"):
            L.rt_debug_lpt_stats.argtypes = [vp, C.POINTER(C.c_int64)]
        if hasattr(L, "rt_debug_wave_stats"):
            L.rt_debug_wave_stats.argtypes = [vp, C.c_int64, vp, C.POINTER(C.c_int64)]
        L.rt_scene_save.argtypes = [vp, C.c_char_p]
        L.rt_frame_download_rgb8.argtypes = [vp, C.c_int64, vp, C.POINTER(C.c_int32)]
        L.rt_write_ppm_rgb8.argtypes = [C.c_char_p, vp, C.c_int32, C.c_int32]
        L.rt_frame_shard_bytes.argtypes = [C.c_int32, C.c_int32, C.c_int32]
        L.rt_trace_closest_normal.argtypes = [vp, C.c_int32, vp, vp, vp, vp, vp, vp]
        L.rt_trace_color.argtypes = [vp, C.c_int32, vp, vp, vp, C.c_int32, vp, vp, vp]
        L.rt_debug_ray.argtypes = [vp, C.POINTER(Camera), vp, C.c_int32, C.c_float, C.c_float, C.c_int32, vp,
                                   C.POINTER(C.c_int32)]
        L.rt_rand_seed.argtypes = [C.POINTER(RandState), C.c_uint32]
        L.rt_rand_seed.restype = None
        L.rt_rand.argtypes = [C.POINTER(RandState)]
        L.rt_rand.restype = C.c_int32
        L.rt_lights_spherical.argtypes = [C.POINTER(Light), C.c_float, C.c_int32, C.POINTER(RandState), C.POINTER(Light)]
        L.rt_lights_spherical.restype = C.c_int32
        L.rt_light_directional.argtypes = [C.POINTER(Camera), C.POINTER(C.c_float * 3), C.POINTER(Light)]
        L.rt_light_directional.restype = None
        L.rt_frame_shard_bytes.restype = C.c_int64
        L.rt_frame_pack_shard_rgb8.argtypes = [vp, vp]
        L.rt_frame_unpack_shards_rgb8.argtypes = [vp, C.c_int32, C.c_int32, C.c_int32, vp, C.c_int32]
        L.rt_scene_load.argtypes = [C.c_char_p, C.POINTER(SceneOpts), C.POINTER(vp)]
        L.rt_box_colors_random.argtypes = [C.c_int32, C.POINTER(RandState), vp]
        L.rt_frame_shard_tiles.argtypes = [C.c_int32, C.c_int32, C.c_int32, C.c_int32, vp, C.c_int32]
        L.rt_frame_shard_tiles.restype = C.c_int32
        L.rt_scene_set_box_colors.argtypes = [vp, vp]
        _lib = L
    return _lib


def _p(a):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


class RTError(RuntimeError):
    pass


def check(rc):
    if rc != 0:
        raise RTError(f"librtamd error {rc}: {lib().rt_last_error().decode()}")


def source_hash(root=None):
    """The hash the Makefile embeds (rt_source_hash), recomputed over the product sources in this tree."""
    import hashlib
    import glob
    pkg = HERE if root is None else os.path.join(root, "ray-tracing-project_amd")
    top = os.path.dirname(pkg)
    files = sorted(glob.glob(os.path.join(pkg, "csrc", "*.hip")) + glob.glob(os.path.join(pkg, "csrc", "*.cpp")) +
                   glob.glob(os.path.join(pkg, "csrc", "*.h")) + [os.path.join(top, "include", "rt", "rt_api.h")],
                   key=lambda p: os.path.relpath(p, top))
    h = hashlib.sha256()
    for f in files:
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def build_identity():
    """{"library": rt_version_string(), "source_hash": embedded, "tree_hash": recomputed, "matches_tree": bool}"""
    emb = lib().rt_source_hash().decode()
    tree = source_hash()
    return {"library": lib().rt_version_string().decode(), "source_hash": emb, "tree_hash": tree,
            "matches_tree": emb == tree}


def device_count():
    return lib().rt_device_count()


class Mesh:
    """Host-side Tucano-semantics mesh (rt_mesh)."""

    def __init__(self, h):
        self.h = h

    @classmethod
    def load_obj(cls, path):
        h = C.c_void_p()
        check(lib().rt_mesh_load_obj(os.fsencode(path), C.byref(h)))
        return cls(h)

    @classmethod
    def from_arrays(cls, v3, faces, materials, vn3=None, groups=None):
        """materials: [nm, 12] (ka3 kd3 ks3 Ns Ni d). groups: [(n_faces, mat_id)]; default one group."""
        v3 = np.ascontiguousarray(v3, np.float32)
        faces = np.ascontiguousarray(faces, np.uint32).reshape(-1)
        mats12 = np.ascontiguousarray(materials, np.float32).reshape(-1, 12)
        if groups is None:
            groups = [(len(faces) // 3, 0 if len(mats12) else -1)]
        gc = np.array([3 * g[0] for g in groups], np.int32)
        gm = np.array([g[1] for g in groups], np.int32)
        mats = (Material * max(len(mats12), 1))()
        for i, m in enumerate(mats12):
            mats[i].ka[:] = list(m[0:3]); mats[i].kd[:] = list(m[3:6]); mats[i].ks[:] = list(m[6:9])
            mats[i].shininess = float(m[9]); mats[i].optical_density = float(m[10]); mats[i].dissolve = float(m[11])
        vn = None if vn3 is None else np.ascontiguousarray(vn3, np.float32)
        h = C.c_void_p()
        check(lib().rt_mesh_from_arrays(len(v3), _p(v3), _p(vn), len(gc), _p(gc), _p(faces), _p(gm), len(mats12),
                                        C.cast(mats, C.c_void_p), C.byref(h)))
        return cls(h)

    def desc(self):
        d = MeshDesc()
        check(lib().rt_mesh_get_desc(self.h, C.byref(d)))
        return d

    def export(self):
        d = self.desc()
        nv, nf, nm = d.n_vertices, d.n_faces, d.n_materials

        def arr(ptr, ctype, shape, dtype):
            n = int(np.prod(shape))
            if n == 0 or not ptr:
                return np.zeros(shape, dtype)
            return np.ctypeslib.as_array(C.cast(ptr, C.POINTER(ctype)), shape=(n,)).reshape(shape).astype(dtype).copy()

        mats = []
        if nm:
            mp = C.cast(d.materials, C.POINTER(Material))
            for i in range(nm):
                m = mp[i]
                mats.append(list(m.ka) + list(m.kd) + list(m.ks) + [m.shininess, m.optical_density, m.dissolve])
        return dict(v4=arr(d.vertices, C.c_float, (nv, 4), np.float32),
                    vn3=arr(d.vertex_normals, C.c_float, (nv, 3), np.float32),
                    fidx=arr(d.face_vertex_ids, C.c_uint32, (nf, 3), np.uint32),
                    fn3=arr(d.face_normals, C.c_float, (nf, 3), np.float32),
                    fmat=arr(d.face_material_ids, C.c_int32, (nf,), np.int32),
                    mats=np.array(mats, np.float32).reshape(-1, 12),
                    M16=np.array(list(d.shape_model_matrix), np.float32))

    def __del__(self):
        if getattr(self, "h", None) and _lib is not None:
            _lib.rt_mesh_destroy(self.h)
            self.h = None


RT_BUILDER_SAH, RT_BUILDER_LBVH_GPU, RT_BUILDER_SBVH, RT_BUILDER_PLOC_GPU, RT_BUILDER_SAH_GPU, RT_BUILDER_SBVH_GPU = 0, 1, 2, 3, 4, 5
RT_BOXES_HOST, RT_BOXES_GPU = 0, 1


def scene_opts(device=-1, min_faces=300, leaf_size=0, frames_in_flight=0, background=None, builder=5,
               box_builder=1, wide_tree=0, devices=None):
    """devices: None = one device (`device`); a list of HIP ordinals (repeats allowed) = a multi-device scene
    (rt_scene_opts.n_devices / devices); RT_DEVICES_ALL = every visible device."""
    o = SceneOpts()
    lib().rt_scene_opts_default(C.byref(o))
    o.builder = builder
    o.box_builder = box_builder
    o.wide_tree = wide_tree
    if background is not None:
        o.background[:] = [float(x) for x in background]
    o.device = device
    o.min_faces = min_faces
    o.leaf_size = leaf_size
    if frames_in_flight:
        o.frames_in_flight = frames_in_flight
    if devices is not None:
        if devices == RT_DEVICES_ALL:
            o.n_devices = RT_DEVICES_ALL
        else:
            devices = list(devices)
            if not 1 <= len(devices) <= RT_MAX_DEVICES:
                raise ValueError(f"1..{RT_MAX_DEVICES} devices")
            o.n_devices = len(devices)
            o.devices[:len(devices)] = [int(d) for d in devices]
    return o


class Scene:
    def __init__(self, mesh, device=-1, min_faces=300, leaf_size=0, frames_in_flight=0, background=None, builder=5,
                 box_builder=1, wide_tree=0, shape_model_matrix=None, devices=None):
        """shape_model_matrix: the desc's getShapeModelMatrix() override (column-major 4x4), e.g. the oracle's
        after Mesh.set_model; default the loader's normalisation. devices: see scene_opts."""
        self.mesh = mesh  # keep the mesh alive (desc borrows its arrays during create)
        self.h = C.c_void_p()
        d = mesh.desc()
        if shape_model_matrix is not None:
            d.shape_model_matrix[:] = [float(x) for x in np.asarray(shape_model_matrix, np.float32).reshape(16)]
        o = scene_opts(device, min_faces, leaf_size, frames_in_flight, background, builder, box_builder, wide_tree, devices)
        check(lib().rt_scene_create(C.byref(d), C.byref(o), C.byref(self.h)))

    def info(self):
        i = SceneInfo()
        check(lib().rt_scene_get_info(self.h, C.byref(i)))
        return {k: getattr(i, k) for k, _ in i._fields_}

    def download(self, W, H, want_hits=False):
        """The last frame (rt_frame_download): rgb [H,W,3], plus face / t when it was rendered with
        RT_FRAME_WRITE_HITS and want_hits is set."""
        rgb = np.zeros((H, W, 3), np.float32)
        face = np.zeros((H, W), np.int32) if want_hits else None
        t = np.zeros((H, W), np.float32) if want_hits else None
        check(lib().rt_frame_download(self.h, W * H, _p(rgb), _p(face), _p(t)))
        return (rgb, face, t) if want_hits else rgb

    def tree_cost(self, k_trav=0.7):
        """rt_debug_tree_cost: SAH cost, node term, triangle term, mean leaf size of the binary tree."""
        out = np.zeros(4, np.float64)
        check(lib().rt_debug_tree_cost(self.h, float(k_trav), _p(out)))
        return dict(sah=float(out[0]), nodes=float(out[1]), tris=float(out[2]), leaf=float(out[3]))

    def record_flags(self):
        """rt_debug_scene_flags: (triangle records, with the safe-normal bit, with the box certificate)."""
        out = np.zeros(3, np.int64)
        check(lib().rt_debug_scene_flags(self.h, _p(out), None, None))
        return tuple(int(x) for x in out)

    def face_flags(self):
        """(per-face OR of the records' flag bits [n_faces] uint32, certificates' object-space origin range)."""
        out = np.zeros(3, np.int64)
        ro = C.c_float(0.0)
        ff = np.zeros(self.info()["n_faces"], np.uint32)
        check(lib().rt_debug_scene_flags(self.h, _p(out), C.byref(ro), _p(ff)))
        return ff, float(ro.value)

    def lpt_stats(self):
        """Longest-first dispatch of lone frames (rt_debug_lpt_stats): {frames, sorts, valid}."""
        out = (C.c_int64 * 3)()
        check(lib().rt_debug_lpt_stats(self.h, out))
        return {"frames": int(out[0]), "sorts": int(out[1]), "valid": bool(out[2])}

    def wave_stats(self):
        """Per-wave counts of the last RT_FRAME_STATS | RT_FRAME_WAVE_STATS frame: uint32 [logical waves, 8]."""
        n = C.c_int64(0)
        check(lib().rt_debug_wave_stats(self.h, 0, None, C.byref(n)))
        out = np.zeros((n.value, 8), np.uint32)
        check(lib().rt_debug_wave_stats(self.h, n.value, _p(out), C.byref(n)))
        return out

    def counters(self, n=16):
        """Raw counters of the last RT_FRAME_STATS frame (rt_debug_counters): int64 [n]."""
        out = (C.c_int64 * n)()
        check(lib().rt_debug_counters(self.h, n, out))
        return [int(x) for x in out]

    def timeline(self):
        """Per-wave records of the last RT_FRAME_TIMELINE frame: uint32 [n_waves, 8] (rt_debug_timeline)."""
        n = C.c_int64(0)
        check(lib().rt_debug_timeline(self.h, 0, None, C.byref(n)))
        out = np.zeros((n.value, 8), np.uint32)
        check(lib().rt_debug_timeline(self.h, n.value, _p(out), C.byref(n)))
        return out

    def download_rgb8(self, W, H):
        """The last frame as writePPMImage's 8-bit values (device conversion); returns (rgb8, exact)."""
        out = np.zeros((H, W, 3), np.uint8)
        ex = C.c_int32(0)
        check(lib().rt_frame_download_rgb8(self.h, W * H, _p(out), C.byref(ex)))
        return out, bool(ex.value)

    def trace_color(self, o, d, lights):
        """traceRay colour (FULL) of arbitrary rays: rgb [n,3], face [n], t [n]"""
        o = np.ascontiguousarray(o, np.float32).reshape(-1, 3)
        d = np.ascontiguousarray(d, np.float32).reshape(-1, 3)
        n = len(o)
        rgb = np.zeros((n, 3), np.float32)
        face = np.zeros(n, np.int32)
        t = np.zeros(n, np.float32)
        L = self._lights(lights)
        check(lib().rt_trace_color(self.h, n, _p(o), _p(d), C.cast(L, C.c_void_p), len(lights), _p(rgb), _p(face), _p(t)))
        return rgb, face, t

    def trace_closest_normal(self, o, d):
        o = np.ascontiguousarray(o, np.float32).reshape(-1, 3)
        d = np.ascontiguousarray(d, np.float32).reshape(-1, 3)
        n = len(o)
        face = np.zeros(n, np.int32)
        t = np.zeros(n, np.float32)
        P = np.zeros((n, 3), np.float32)
        N = np.zeros((n, 3), np.float32)
        check(lib().rt_trace_closest_normal(self.h, n, _p(o), _p(d), _p(face), _p(t), _p(P), _p(N)))
        return face, t, P, N

    def debug_ray(self, cam, lights, mouse_x, mouse_y, max_depth=2):
        """createDebugRay: [(origin3, direction3, length, color3), ...]"""
        segs = (RaySegment * max_depth)()
        n = C.c_int32(0)
        L = self._lights(lights)
        check(lib().rt_debug_ray(self.h, C.byref(cam), C.cast(L, C.c_void_p), len(lights), mouse_x, mouse_y, max_depth,
                                 segs, C.byref(n)))
        return [(np.array(g.origin, np.float32), np.array(g.direction, np.float32), np.float32(g.length),
                 np.array(g.color, np.float32)) for g in segs[: n.value]]

    def pack_shard_rgb8(self, dst_device_ptr):
        """This rank's tiles of the last frame, 8-bit, into device memory (rt_frame_pack_shard_rgb8)."""
        check(lib().rt_frame_pack_shard_rgb8(self.h, C.c_void_p(dst_device_ptr)))

    def save(self, path):
        """Binary scene cache (rt_scene_save)."""
        check(lib().rt_scene_save(self.h, os.fsencode(path)))

    @classmethod
    def load(cls, path, device=-1, frames_in_flight=0, wide_tree=0, devices=None):
        """Scene from a binary cache (rt_scene_load): no OBJ parsing, no builds."""
        self = cls.__new__(cls)
        self.mesh = None
        self.h = C.c_void_p()
        o = scene_opts(device, 300, 0, frames_in_flight, wide_tree=wide_tree, devices=devices)
        check(lib().rt_scene_load(os.fsencode(path), C.byref(o), C.byref(self.h)))
        return self

    def validate_bvh(self):
        """Host check of both trees (containment + exact leaf cover); returns the info counters."""
        info = np.zeros(7, np.int64)
        rc = lib().rt_debug_validate_bvh(self.h, _p(info))
        keys = ["nodes2", "depth2", "nodes4", "depth4", "covered2", "covered4", "violations"]
        out = dict(zip(keys, (int(x) for x in info)))
        out["ok"] = rc == 0
        return out

    def set_box_colors(self, colors=None):
        """rt_scene_set_box_colors: colours [n_ref_boxes, 3] of RT_MODE_BOX_COLORS (None = the reference's
        setRandomColor sequence of a fresh process)."""
        c = None if colors is None else np.ascontiguousarray(colors, np.float32).reshape(-1, 3)
        if c is not None and len(c) != self.info()["n_ref_boxes"]:
            raise ValueError("one colour per reference box")
        check(lib().rt_scene_set_box_colors(self.h, _p(c)))

    def ref_boxes(self):
        inf = self.info()
        nb, nf = inf["n_ref_boxes"], inf["n_faces"]
        b6 = np.zeros((nb, 6), np.float32)
        cnt = np.zeros(nb, np.int32)
        order = np.zeros(nf, np.int32)
        check(lib().rt_scene_ref_boxes(self.h, _p(b6), _p(cnt), _p(order)))
        return b6, cnt, order

    @staticmethod
    def _lights(lights):
        """[(pos3, color3) | (vec3, color3, kind)] -> rt_light array"""
        arr = (Light * max(len(lights), 1))()
        for i, l in enumerate(lights):
            arr[i].position[:] = list(l[0])
            arr[i].color[:] = list(l[1])
            arr[i].kind = l[2] if len(l) > 2 else RT_LIGHT_POINT
        return arr

    def render(self, cam, lights, W, H, mode=RT_MODE_PRIMARY, shard=(0, 1), flags=0, want_hits=False, max_depth=0):
        """rt_render: rgb [H,W,3] (+ face, t with want_hits) and the stats. max_depth: traceRay's recursion
        limit (0 = the mode's own: PRIMARY 1, FULL 2)."""
        fr = Frame(W, H, mode, shard[0], shard[1], flags | (RT_FRAME_WRITE_HITS if want_hits else 0), max_depth)
        rgb = np.zeros((H, W, 3), np.float32)
        st = Stats()
        L = self._lights(lights)
        check(lib().rt_render(self.h, C.byref(cam), C.cast(L, C.c_void_p), len(lights), C.byref(fr), _p(rgb),
                              C.byref(st)))
        if want_hits:
            face = np.zeros((H, W), np.int32)
            t = np.zeros((H, W), np.float32)
            check(lib().rt_frame_download(self.h, W * H, None, _p(face), _p(t)))
            return rgb, face, t, st.as_dict()
        return rgb, st.as_dict()

    def render_async(self, cam, lights, W, H, mode=RT_MODE_PRIMARY, shard=(0, 1), flags=0, max_depth=0):
        self._keep = self._lights(lights)
        fr = Frame(W, H, mode, shard[0], shard[1], flags, max_depth)
        check(lib().rt_render_async(self.h, C.byref(cam), C.cast(self._keep, C.c_void_p), len(lights), C.byref(fr)))

    def synchronize(self):
        st = Stats()
        check(lib().rt_synchronize(self.h, C.byref(st)))
        return st.as_dict()

    def synchronize_devices(self):
        """rt_synchronize_devices: (totals over the devices, [per-device stats])."""
        st = Stats()
        per = (Stats * RT_MAX_DEVICES)()
        n = lib().rt_synchronize_devices(self.h, C.byref(st), RT_MAX_DEVICES, per)
        if n < 0:
            check(n)
        return st.as_dict(), [per[k].as_dict() for k in range(n)]

    def trace_closest(self, o, d):
        o = np.ascontiguousarray(o, np.float32).reshape(-1, 3)
        d = np.ascontiguousarray(d, np.float32).reshape(-1, 3)
        n = len(o)
        face = np.zeros(n, np.int32)
        t = np.zeros(n, np.float32)
        P = np.zeros((n, 3), np.float32)
        check(lib().rt_trace_closest(self.h, n, _p(o), _p(d), _p(face), _p(t), _p(P)))
        return face, t, P

    def trace_shadow(self, P, L):
        P = np.ascontiguousarray(P, np.float32).reshape(-1, 3)
        L = np.ascontiguousarray(L, np.float32).reshape(-1, 3)
        out = np.zeros(len(P), np.int32)
        check(lib().rt_trace_shadow(self.h, len(P), _p(P), _p(L), _p(out)))
        return out

    def __del__(self):
        if getattr(self, "h", None) and _lib is not None:
            _lib.rt_scene_destroy(self.h)
            self.h = None


def record_layout(n_nodes, n_tris, n_wide):
    """rt_debug_record_layout: (allocation bytes or 0, wide copies' byte offset or 0 = wide tree dropped)."""
    out = np.zeros(2, np.int64)
    check(lib().rt_debug_record_layout(n_nodes, n_tris, n_wide, _p(out)))
    return int(out[0]), int(out[1])


def flycam(W, H, dx=0.0, dy=0.0, dz=0.0):
    c = Camera()
    lib().rt_camera_flycam(W, H, dx, dy, dz, C.byref(c))
    return c


FLYCAM_SPEED = np.float32(0.05)  # Tucano::Flycamera::speed (flycamera.hpp:107)
WASD_STEP = 0.2                  # Flyscene::simulate: a held key moves 0.2 per frame (flyscene.cpp:116-127)


def flycam_tv(W, H, tv):
    """The Flycamera of Flyscene::initialize (fovy 60, aspect W/H, viewport) whose translation_vector is tv
    (float32[3]), after updateViewMatrix at zero rotation (flycamera.hpp:166-191): view = T(0,0,-2) * T(tv), i.e.
    the view translation (0 + tv.x, 0 + tv.y, -2 + tv.z) in float -- what rt_camera_flycam computes for one
    translate() from the default pose (tests/test_host.py holds the two equal)."""
    tv = np.asarray(tv, np.float32)
    c = Camera()
    m = np.eye(4, dtype=np.float32).reshape(-1)  # column-major; identity linear part
    m[12] = np.float32(0.0) + tv[0]
    m[13] = np.float32(0.0) + tv[1]
    m[14] = np.float32(-2.0) + tv[2]
    for k in range(16):
        c.view_matrix[k] = float(m[k])
    c.viewport[:] = [0.0, 0.0, float(W), float(H)]
    c.fovy = 60.0
    c.aspect_ratio = float(np.float32(W) / np.float32(H))
    return c


class CameraPath:
    """The camera of the reference's interactive loop (main.cpp:123-130: paintGL, then simulate) with keys held:
    every frame Flyscene::simulate calls flycamera.translate(dx, dy, dz) with +-0.2 per held key
    (flyscene.cpp:116-127), and Flycamera::translate adds yaw * (-dx, -dy, dz) * speed to its translation vector
    in float (flycamera.hpp:196-202; yaw = identity at rotation_Y_axis 0): 0.01 scene units per axis per frame.
    The path holds W (forward) and D (strafe) and turns each round -- W <-> S every `period_z` frames, D <-> A every
    `period_x` -- so the pose stays within 0.4 x 0.25 units of the start while it changes every frame. Starts
    from the bench's pose translate(dx0, dy0, dz0) (eye (0, 0, 1) for dz0 = 20)."""

    def __init__(self, W, H, dx0=0.0, dy0=0.0, dz0=20.0, period_z=40, period_x=25):
        self.W, self.H = W, H
        self.i = 0
        self.pz, self.px = period_z, period_x
        self.tv = np.zeros(3, np.float32)
        self._move(dx0, dy0, dz0)

    def _move(self, dx, dy, dz):
        v = np.array([-dx, -dy, dz], np.float32)          # yaw * Vector3f(-dx, -dy, dz): identity rotation
        self.tv = (self.tv + v * FLYCAM_SPEED).astype(np.float32)

    def keys(self, i):
        """(dx, dy, dz) of frame i's simulate(): D / A and W / S alternating."""
        dz = WASD_STEP if (i // self.pz) % 2 == 0 else -WASD_STEP
        dx = WASD_STEP if (i // self.px) % 2 == 0 else -WASD_STEP
        return dx, 0.0, dz

    def camera(self):
        return flycam_tv(self.W, self.H, self.tv)

    def next(self):
        """The camera for the next frame: the current pose is rendered, then simulate() moves it."""
        c = self.camera()
        self._move(*self.keys(self.i))
        self.i += 1
        return c

    def take(self, n):
        return [self.next() for _ in range(n)]


def generate_soup(n_tris, seed=12345):
    v = np.zeros((3 * n_tris, 3), np.float32)
    lib().rt_generate_soup(n_tris, seed, _p(v))
    return v


def write_ppm(path, rgb):
    rgb = np.ascontiguousarray(rgb, np.float32)
    H, W = rgb.shape[:2]
    check(lib().rt_write_ppm(os.fsencode(path), _p(rgb), W, H))


def set_variant(v):
    """Kernel-variant override (A/B and tests); returns the previous value."""
    return lib().rt_debug_set_variant(int(v))


class Rand:
    """glibc rand() (the reference's unseeded rand(): seed 1)"""

    def __init__(self, seed=1):
        self.st = RandState()
        lib().rt_rand_seed(C.byref(self.st), seed)

    def __call__(self):
        return lib().rt_rand(C.byref(self.st))


def shard_tiles(W, H, k, n):
    """rt_frame_shard_tiles: the (tile x, tile y) 16x16 tiles shard k of n renders, in slot order."""
    m = lib().rt_frame_shard_tiles(W, H, k, n, None, 0)
    out = np.zeros((max(m, 1), 2), np.int32)
    lib().rt_frame_shard_tiles(W, H, k, n, _p(out), m)
    return [tuple(map(int, t)) for t in out[:m]]


def shard_mask(W, H, k, n):
    """[H, W] bool: the pixels shard k of n renders."""
    m = np.zeros((H, W), bool)
    for tx, ty in shard_tiles(W, H, k, n):
        m[ty * 16:ty * 16 + 16, tx * 16:tx * 16 + 16] = True
    return m


def box_colors_random(n_boxes, rng=None):
    """BoundingBox::setRandomColor for n_boxes boxes in creation order from rng (None = seed 1)."""
    out = np.zeros((n_boxes, 3), np.float32)
    check(lib().rt_box_colors_random(n_boxes, C.byref(rng.st) if rng else None, _p(out)))
    return out


def spherical_light(pos, color, radius, n_points, rng=None):
    """Flyscene::sphericalLight + addLight('s'): n_points jittered lights then the centre, as
    [(pos3, color3), ...] point lights."""
    c = Light()
    c.position[:] = list(pos)
    c.color[:] = list(color)
    out = (Light * (n_points + 1))()
    n = lib().rt_lights_spherical(C.byref(c), radius, n_points, C.byref(rng.st) if rng else None, out)
    if n < 0:
        check(n)
    return [(tuple(out[i].position), tuple(out[i].color)) for i in range(n)]


def directional_light(cam, color):
    """addLight('d'): (vector3, color3, RT_LIGHT_DIRECTIONAL) with the reference's stored vector."""
    col = (C.c_float * 3)(*color)
    out = Light()
    lib().rt_light_directional(C.byref(cam), C.byref(col), C.byref(out))
    return (tuple(out.position), tuple(out.color), RT_LIGHT_DIRECTIONAL)


def shard_bytes(W, H, n):
    return int(lib().rt_frame_shard_bytes(W, H, n))


def unpack_shards_rgb8(packed_ptr, n, W, H, frame_ptr, device=-1):
    check(lib().rt_frame_unpack_shards_rgb8(C.c_void_p(packed_ptr), n, W, H, C.c_void_p(frame_ptr), device))


def write_ppm_rgb8(path, rgb8):
    rgb8 = np.ascontiguousarray(rgb8, np.uint8)
    check(lib().rt_write_ppm_rgb8(os.fsencode(path), _p(rgb8), rgb8.shape[1], rgb8.shape[0]))


def debug_math(op, inp, n, out_len, device=False):
    out = np.zeros(n * out_len, np.float32)
    inp = np.ascontiguousarray(inp, np.float32)
    f = lib().rt_debug_math_device if device else lib().rt_debug_math_host
    check(f(op, n, _p(inp), _p(out)))
    return out


DEFAULT_LIGHTS = [((-0.5, 2.0, 3.0), (1.0, 1.0, 1.0))]  # flyscene.cpp:37
SOUP_MATERIAL = [0.1, 0.1, 0.1, 0.7, 0.7, 0.7, 0.2, 0.2, 0.2, 16.0, 1.0, 1.0]  # C3/C4


def soup_mesh(n_tris, seed=12345):
    v = generate_soup(n_tris, seed)
    f = np.arange(3 * n_tris, dtype=np.uint32).reshape(-1, 3)
    return Mesh.from_arrays(v, f, np.array([SOUP_MATERIAL], np.float32)), v, f
