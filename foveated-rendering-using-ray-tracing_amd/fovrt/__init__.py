"""fovrt — Python mirror of the reference's renderer classes over the libfovrt C ABI.

The reference drives its hot path from C++ (FR/main.cpp:152-462) through the classes
``PathTracer``, ``JumpFlooding``, ``SibsonInterpolation``, ``PullPushInterpolation``, ``ATrous`` and
``Camera``.  This module exposes the same names, method names and argument order on top of
``include/fovrt.h`` (ctypes, no torch types), so tests and the benchmark read like the reference's
frame loop.  GL texture handles become fr_buffer_id integers; ``get_texture`` returns the buffer id
and ``read`` copies a buffer to a numpy array.

Nothing here computes pixels: every stage runs in the HIP kernels of libfovrt.so.  Importing this
module does not touch the GPU; creating a ``PathTracer`` does, and fails loudly (FovrtError) if the
library or a device is missing.
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass

import numpy as np

_PKG_DIR = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(os.path.dirname(_PKG_DIR), "libfovrt.so")
REPO_ROOT = os.path.dirname(os.path.dirname(_PKG_DIR))
DEFAULT_ASSET_DIR = os.path.join(REPO_ROOT, "assets")

ABI_VERSION = 2  # FOVRT_ABI_VERSION of include/fovrt.h this mirror is written against
GROUP_MAX_VIEW_RANKS = 16
# fr_status
FR_OK, FR_E_INVALID, FR_E_HIP, FR_E_NOMEM, FR_E_IO, FR_E_STATE, FR_E_UNSUPPORTED = 0, -1, -2, -3, -4, -5, -6
# scenes / masks
SCENE_BOX, SCENE_BUNNY, SCENE_VOKSELIA = 0, 1, 2
MASK_SALIENCY, MASK_LOGPOLAR, MASK_UNIFORM2X2, MASK_ALL, MASK_LOGPOLAR_SIGNED = 0, 1, 2, 3, 4
# fr_set_pipeline_mode
PIPELINE_THROUGHPUT, PIPELINE_LATENCY = 0, 1
SCENES = {"box": SCENE_BOX, "bunny": SCENE_BUNNY, "vokselia": SCENE_VOKSELIA}
MASKS = {"saliency": MASK_SALIENCY, "logpolar": MASK_LOGPOLAR, "uniform": MASK_UNIFORM2X2, "all": MASK_ALL,
         "logpolar10": MASK_LOGPOLAR_SIGNED}


class TextureName:
    """PathTracer::TextureName (FR/PathTracer.h:13-31) plus the reconstruction outputs."""
    POSITION, NORMAL, DEPTH, DIFFUSE, WEIGHT, THREAD, HISTORY, SHADING, EXTRA = range(9)
    JFA_COORD, JFA_COLOR, SIBSON, PULLPUSH, ATROUS, DEPTH_CACHE, HISTORY_CACHE, MASK = range(9, 17)
    LOGPOLAR, LOGPOLAR_INVERSE, GCLASS = 17, 18, 19


class FovrtError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"fovrt error {code}: {msg}")
        self.code = code


class fr_config(C.Structure):
    _fields_ = [("abi_version", C.c_int), ("width", C.c_int), ("height", C.c_int), ("scene", C.c_int),
                ("mask_mode", C.c_int),
                ("spp", C.c_int), ("diffuse_max_depth", C.c_int), ("refraction_max_depth", C.c_int),
                ("light_power", C.c_float), ("optimize", C.c_int), ("atrous_iterations", C.c_int),
                ("write_extra", C.c_int), ("device", C.c_int), ("texture_mode", C.c_int), ("detail", C.c_int),
                ("mesh_mode", C.c_int), ("bvh_builder", C.c_int), ("sibson_mode", C.c_int),
                ("asset_dir", C.c_char_p)]


class fr_camera(C.Structure):
    _fields_ = [("eye", C.c_float * 3), ("prev_eye", C.c_float * 3), ("inv_vp", C.c_float * 16),
                ("prev_vp", C.c_float * 16), ("up", C.c_float * 3), ("target", C.c_float * 3),
                ("gaze", C.c_float * 2)]


class fr_camera_pose(C.Structure):
    _fields_ = [("pos", C.c_float * 3), ("rot", C.c_float * 4), ("fovy_deg", C.c_float),
                ("znear", C.c_float), ("zfar", C.c_float), ("aspect", C.c_float)]


class fr_buffer_view(C.Structure):
    _fields_ = [("device_ptr", C.c_void_p), ("width", C.c_int), ("height", C.c_int),
                ("pitch_bytes", C.c_size_t), ("bytes", C.c_size_t), ("format", C.c_int)]


class fr_stats(C.Structure):
    _fields_ = [(n, C.c_uint64) for n in ("gbuffer_primary", "primary", "shadow", "diffuse_bounce", "mirror",
                                          "refraction", "reflection", "truncated", "overflow", "segments")] + \
                [("diag", C.c_uint64 * 6)]


class fr_frame_timing(C.Structure):
    _fields_ = [(n, C.c_float) for n in ("geometry_ms", "sampling_ms", "optimize_ms", "shading_ms", "jfa_ms",
                                         "sibson_ms", "pullpush_ms", "atrous_ms", "total_ms")] + \
               [("ray_count", C.c_uint32), ("shade_paths_ms", C.c_float)]


class fr_stage_times(C.Structure):
    _fields_ = [("frames", C.c_uint32), ("shading_ms", C.c_double), ("shade_paths_ms", C.c_double)]


class fr_group_config(C.Structure):
    _fields_ = [("views", C.c_int), ("tile", C.c_int), ("split_recon", C.c_int), ("moving_camera", C.c_int),
                ("composite", C.c_int), ("recon_cost", C.c_float * 2), ("weights", C.c_float * GROUP_MAX_VIEW_RANKS),
                ("sample_sum", C.c_int), ("front_local", C.c_int),
                ("jfa_ranks", C.c_int)]


class fr_scene_arrays(C.Structure):
    _fields_ = [("num_tris", C.c_int), ("pos", C.POINTER(C.c_float)), ("nrm", C.POINTER(C.c_float)),
                ("uv", C.POINTER(C.c_float)), ("flags", C.POINTER(C.c_int32)), ("num_materials", C.c_int),
                ("materials", C.POINTER(C.c_int32)), ("num_textures", C.c_int), ("tex_dims", C.POINTER(C.c_int32)),
                ("tex_data", C.POINTER(C.POINTER(C.c_float))), ("envmap", C.c_int), ("light", C.c_float * 15),
                ("bbox", C.c_float * 6), ("bvh_nodes", C.c_int), ("bvh_depth", C.c_int),
                ("bvh_max_stack", C.c_int)]


# exported symbols and their signatures (kept in sync with include/fovrt.h)
_SIGS = {
    "fr_config_default": [C.POINTER(fr_config)],
    "fr_version": [],
    "fr_abi_version": [],
    "fr_create": [C.POINTER(fr_config), C.POINTER(C.c_void_p)],
    "fr_destroy": [C.c_void_p],
    "fr_last_error": [C.c_void_p],
    "fr_camera_look_at": [C.POINTER(fr_camera_pose), C.POINTER(C.c_float), C.POINTER(C.c_float)],
    "fr_camera_matrices": [C.POINTER(fr_camera_pose), C.POINTER(C.c_float), C.POINTER(C.c_float)],
    "fr_camera_uniforms": [C.POINTER(fr_camera_pose), C.POINTER(fr_camera_pose), C.c_int, C.c_int,
                           C.POINTER(fr_camera)],
    "fr_preset_camera": [C.c_int, C.POINTER(C.c_float), C.POINTER(C.c_float)],
    "fr_set_camera": [C.c_void_p, C.POINTER(fr_camera)],
    "fr_set_light_power": [C.c_void_p, C.c_float],
    "fr_set_diffuse_max_depth": [C.c_void_p, C.c_int],
    "fr_reset_accumulation": [C.c_void_p],
    "fr_accum_frame": [C.c_void_p, C.POINTER(C.c_uint32)],
    "fr_geometry_launch": [C.c_void_p, C.POINTER(C.c_float)],
    "fr_sampling_launch": [C.c_void_p, C.POINTER(C.c_float)],
    "fr_optimize_launch": [C.c_void_p, C.POINTER(C.c_float)],
    "fr_shading_launch": [C.c_void_p, C.POINTER(C.c_float)],
    "fr_ray_count": [C.c_void_p, C.POINTER(C.c_uint32)],
    "fr_gaze_target": [C.c_void_p, C.POINTER(C.c_float)],
    "fr_jfa_render": [C.c_void_p, C.c_int, C.POINTER(C.c_uint64)],
    "fr_sibson_render": [C.c_void_p, C.POINTER(C.c_uint64)],
    "fr_pullpush_render": [C.c_void_p, C.c_int, C.POINTER(C.c_uint64)],
    "fr_atrous_render": [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.POINTER(C.c_uint64)],
    "fr_logpolar_render": [C.c_void_p, C.c_int, C.POINTER(C.c_uint64)],
    "fr_set_gaze": [C.c_void_p, C.c_double, C.c_double, C.c_int],
    "fr_reset_gaze": [C.c_void_p],
    "fr_composite_views": [C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_size_t],
    "fr_frame": [C.c_void_p, C.POINTER(fr_frame_timing)],
    "fr_set_recon_chains": [C.c_void_p, C.c_int],
    "fr_set_pipeline_mode": [C.c_void_p, C.c_int],
    "fr_set_sample_sum": [C.c_void_p, C.c_int],
    "fr_set_front_local": [C.c_void_p, C.c_int],
    "fr_shard_unpack_active_enqueue": [C.c_void_p, C.c_void_p, C.c_size_t, C.c_uint32, C.c_uint32],
    "fr_trace_frame": [C.c_void_p, C.POINTER(fr_frame_timing)],
    "fr_reconstruct_frame": [C.c_void_p, C.POINTER(fr_frame_timing)],
    "fr_set_shard": [C.c_void_p, C.c_int, C.c_int, C.c_int],
    "fr_set_shard_ex": [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int],
    "fr_set_shard_plan": [C.c_void_p, C.c_int, C.c_int, C.c_int, C.POINTER(C.c_uint8), C.c_size_t],
    "fr_shard_plan": [C.c_int, C.c_int, C.c_int, C.c_int, C.POINTER(C.c_float), C.POINTER(C.c_uint8), C.c_size_t],
    "fr_shard_counts": [C.c_void_p, C.POINTER(C.c_uint32), C.c_int],
    "fr_shard_pack_active": [C.c_void_p, C.c_void_p, C.c_size_t, C.c_uint32, C.POINTER(C.c_uint32)],
    "fr_shard_unpack_active": [C.c_void_p, C.c_void_p, C.c_size_t, C.c_uint32, C.c_uint32],
    "fr_shard_texels": [C.c_void_p, C.POINTER(C.c_size_t)],
    "fr_shard_pack": [C.c_void_p, C.c_int, C.c_void_p, C.c_size_t],
    "fr_shard_unpack": [C.c_void_p, C.c_int, C.c_int, C.c_void_p, C.c_size_t],
    "fr_synchronize": [C.c_void_p],
    "fr_get_buffer": [C.c_void_p, C.c_int, C.POINTER(fr_buffer_view)],
    "fr_read_buffer": [C.c_void_p, C.c_int, C.c_void_p, C.c_size_t],
    "fr_write_buffer": [C.c_void_p, C.c_int, C.c_void_p, C.c_size_t],
    "fr_copy_buffer": [C.c_void_p, C.c_int, C.c_void_p, C.c_size_t],
    "fr_snapshot_bytes": [C.c_void_p, C.POINTER(C.c_size_t)],
    "fr_snapshot": [C.c_void_p, C.c_void_p, C.c_size_t],
    "fr_restore": [C.c_void_p, C.c_void_p, C.c_size_t],
    "fr_rebuild_bvh": [C.c_void_p, C.POINTER(C.c_float)],
    "fr_set_positions": [C.c_void_p, C.POINTER(C.c_float), C.c_size_t],
    "fr_get_stats": [C.c_void_p, C.POINTER(fr_stats)],
    "fr_reset_stats": [C.c_void_p],
    "fr_kernel_timing": [C.c_void_p, C.c_int],
    "fr_kernel_times": [C.c_void_p, C.POINTER(fr_stage_times)],
    "fr_frame_clock": [C.c_void_p, C.c_int],
    "fr_frame_clock_read": [C.c_void_p, C.POINTER(C.c_float), C.POINTER(C.c_float), C.c_int, C.POINTER(C.c_int),
                            C.POINTER(C.c_int)],
    "fr_scene_export": [C.c_void_p, C.POINTER(fr_scene_arrays)],
    "fr_scene_create": [C.POINTER(fr_config), C.POINTER(C.c_void_p)],
    "fr_scene_get_arrays": [C.c_void_p, C.POINTER(fr_scene_arrays)],
    "fr_scene_destroy": [C.c_void_p],
    "fr_group_config_default": [C.POINTER(fr_group_config)],
    "fr_rccl_unique_id": [C.c_void_p],
    "fr_rccl_comm_init": [C.c_void_p, C.c_int, C.c_int, C.c_int, C.POINTER(C.c_void_p)],
    "fr_rccl_comm_destroy": [C.c_void_p],
    "fr_group_create": [C.POINTER(C.c_void_p), C.c_int, C.c_void_p, C.POINTER(fr_group_config), C.POINTER(C.c_void_p)],
    "fr_group_frame": [C.c_void_p, C.POINTER(fr_frame_timing)],
    "fr_group_composite": [C.c_void_p, C.c_void_p, C.c_size_t],
    "fr_group_rank_info": [C.c_void_p, C.c_int, C.POINTER(C.c_int), C.POINTER(C.c_int), C.POINTER(C.c_int),
                           C.POINTER(C.c_int)],
    "fr_group_tile_owners": [C.c_void_p, C.c_void_p, C.c_size_t],
    "fr_group_output_ranks": [C.c_void_p, C.c_int, C.POINTER(C.c_int), C.POINTER(C.c_int)],
    "fr_group_plan": [C.c_int, C.c_int, C.c_int, C.POINTER(fr_group_config), C.c_void_p, C.c_size_t],
    "fr_group_synchronize": [C.c_void_p],
    "fr_group_destroy": [C.c_void_p],
    "fr_group_last_error": [],
}

_lib = None


def load_library(path: str | None = None):
    """Loads libfovrt.so (raises FovrtError if it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    path = path or os.environ.get("FOVRT_LIB") or LIB_PATH  # FOVRT_LIB: a diagnostic build of the same ABI
    if not os.path.exists(path):
        raise FovrtError(FR_E_STATE, f"{path} not built: run __graft_entry__.build() or make -C "
                                     f"foveated-rendering-using-ray-tracing_amd")
    lib = C.CDLL(path)
    older = path != LIB_PATH and os.environ.get("FOVRT_LIB_OLDER") == "1"  # A/B against an older build
    for name, args in _SIGS.items():
        if older and not hasattr(lib, name):
            continue
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = C.c_char_p if name in ("fr_version", "fr_last_error", "fr_group_last_error") else C.c_int
    if lib.fr_abi_version() != ABI_VERSION:
        raise FovrtError(FR_E_STATE, f"{path}: ABI version {lib.fr_abi_version()}, this mirror expects {ABI_VERSION}")
    _lib = lib
    return lib


def _f(arr, n):
    return (C.c_float * n)(*[float(v) for v in arr])


# ------------------------------------------------------------------------------------------
# Camera (FR/Camera.cpp): pose state on the host, matrices from the C ABI's glm restatement.
# ------------------------------------------------------------------------------------------
class Camera:
    PM_Perspective = 0

    def __init__(self):
        self.pos = np.zeros(3, np.float32)
        self.rot = np.array([1, 0, 0, 0], np.float32)  # glm::quat (w, x, y, z); FR/Camera.cpp:12 is (0,0,0,1) xyzw
        self.fovy, self.znear, self.zfar = 45.0, 0.01, 100.0
        self.aspect = 1.0
        self.screen = (1, 1)
        self.target = np.zeros(3, np.float32)
        self.prev = None  # previous pose (setPrevState); None -> same as current

    def setPosition(self, p):
        self.pos = np.asarray(p, np.float32).copy()

    def setRotation(self, q):
        self.rot = np.asarray(q, np.float32).copy()

    def setTarget(self, t):
        self.target = np.asarray(t, np.float32).copy()

    def setProjectMode(self, mode, fovy, n, f):
        self.fovy, self.znear, self.zfar = float(fovy), float(n), float(f)

    def setScreen(self, screen):
        self.screen = (int(screen[0]), int(screen[1]))

    def setViewport(self, vp):
        self.aspect = np.float32(vp[2]) / np.float32(vp[3])

    def lookAt(self, target, up=(0.0, 1.0, 0.0)):
        lib = load_library()
        pose = self._pose()
        lib.fr_camera_look_at(C.byref(pose), _f(target, 3), _f(up, 3))
        self.rot = np.array(pose.rot[:], np.float32)
        self.target = np.asarray(target, np.float32).copy()

    def _pose(self, which=None):
        p = fr_camera_pose()
        src = which or (self.pos, self.rot, self.fovy, self.znear, self.zfar, self.aspect)
        p.pos[:] = [float(v) for v in src[0]]
        p.rot[:] = [float(v) for v in src[1]]
        p.fovy_deg, p.znear, p.zfar, p.aspect = float(src[2]), float(src[3]), float(src[4]), float(src[5])
        return p

    def getVMat(self):
        return self._matrices()[0]

    def getPMat(self):
        return self._matrices()[1]

    def _matrices(self):
        lib = load_library()
        v, p = (C.c_float * 16)(), (C.c_float * 16)()
        lib.fr_camera_matrices(C.byref(self._pose()), v, p)
        return np.array(v[:], np.float32).reshape(4, 4), np.array(p[:], np.float32).reshape(4, 4)

    def setPrevState(self):
        self.prev = (self.pos.copy(), self.rot.copy(), self.fovy, self.znear, self.zfar, self.aspect)

    def uniforms(self, width, height) -> fr_camera:
        lib = load_library()
        cam = fr_camera()
        cur = self._pose()
        prev = self._pose(self.prev) if self.prev is not None else cur
        rc = lib.fr_camera_uniforms(C.byref(cur), C.byref(prev), int(width), int(height), C.byref(cam))
        if rc:
            raise FovrtError(rc, "fr_camera_uniforms")
        return cam

    @staticmethod
    def preset(scene, width, height):
        """The reference's camera set-up (FR/main.cpp:179-209) for a scene preset."""
        lib = load_library()
        eye, tgt = (C.c_float * 3)(), (C.c_float * 3)()
        lib.fr_preset_camera(int(scene), eye, tgt)
        cam = Camera()
        cam.setRotation((1, 0, 0, 0))
        cam.setPosition(eye[:])
        cam.lookAt(tgt[:])
        cam.setProjectMode(Camera.PM_Perspective, 45, 0.1, 500.1)
        cam.setScreen((width, height))
        cam.setViewport((0, 0, width, height))
        return cam


@dataclass
class Config:
    width: int = 1024
    height: int = 1024
    scene: int = SCENE_BUNNY
    mask_mode: int = MASK_SALIENCY
    spp: int = 1
    diffuse_max_depth: int = 1
    refraction_max_depth: int = 16
    light_power: float = 810.0
    optimize: int = 1
    atrous_iterations: int = 1
    write_extra: int = 1
    device: int = 0
    texture_mode: int = 0
    detail: int = 0
    mesh_mode: int = 0  # 0: .obj meshes where present, else procedural; 1: procedural; 2: .obj required
    bvh_builder: int = 0  # 0: host binned SAH; 1: GPU LBVH (k_bvh.hip)
    sibson_mode: int = 0  # 0: run form (prefix sums, ~1e-6 of the per-tap sum); 1: per tap, bit-exact
    asset_dir: str = DEFAULT_ASSET_DIR

    def to_c(self) -> fr_config:
        c = fr_config()
        for f in fr_config._fields_:
            name = f[0]
            if name == "asset_dir":
                c.asset_dir = self.asset_dir.encode()
            elif name == "abi_version":
                c.abi_version = ABI_VERSION
            else:
                setattr(c, name, getattr(self, name))
        return c


# ------------------------------------------------------------------------------------------
# PathTracer (FR/PathTracer.h:73-94)
# ------------------------------------------------------------------------------------------
class PathTracer:
    def __init__(self, config: Config | None = None):
        self.config = config or Config()
        self._ctx = None

    # bool initialize(int w, int h)
    def initialize(self, width=None, height=None):
        if self._ctx is not None:
            return False  # FR/PathTracer.cpp:43-45
        lib = load_library()
        if width is not None:
            self.config.width, self.config.height = int(width), int(height)
        self._cfg = self.config.to_c()  # keep asset_dir bytes alive
        ctx = C.c_void_p()
        rc = lib.fr_create(C.byref(self._cfg), C.byref(ctx))
        if rc:
            raise FovrtError(rc, lib.fr_last_error(None).decode())
        self._ctx = ctx
        return True

    def __del__(self):
        self.destroy()

    def destroy(self):
        # a group over this context goes first (fr_group_destroy reads its contexts; under garbage
        # collection of a cycle the tracers' finalisers can run before the group's)
        for grp in getattr(self, "_groups", ()):
            grp.destroy()  # (strong references: weak ones are cleared before a cycle's finalisers run)
        self._groups = []
        if getattr(self, "_ctx", None) is not None and _lib is not None:
            _lib.fr_destroy(self._ctx)
            self._ctx = None

    def _check(self, rc):
        if rc:
            raise FovrtError(rc, _lib.fr_last_error(self._ctx).decode())

    @property
    def width(self):
        return self.config.width

    @property
    def height(self):
        return self.config.height

    def init_camera(self, camera: Camera):
        self.update_optix_variables(camera)

    def update_optix_variables(self, camera: Camera):
        cam = camera.uniforms(self.width, self.height)
        self._check(_lib.fr_set_camera(self._ctx, C.byref(cam)))

    def set_camera_uniforms(self, cam: fr_camera):
        self._check(_lib.fr_set_camera(self._ctx, C.byref(cam)))

    def _launch(self, fn):
        ms = C.c_float()
        self._check(fn(self._ctx, C.byref(ms)))
        return ms.value

    def geometry_launch(self):
        return self._launch(_lib.fr_geometry_launch)

    def sampling_launch(self):
        return self._launch(_lib.fr_sampling_launch)

    def optimize_launch(self):
        return self._launch(_lib.fr_optimize_launch)

    def shading_launch(self):
        return self._launch(_lib.fr_shading_launch)

    @property
    def m_accumFrame(self):
        v = C.c_uint32()
        self._check(_lib.fr_accum_frame(self._ctx, C.byref(v)))
        return v.value

    def reset_accumulation(self):
        self._check(_lib.fr_reset_accumulation(self._ctx))

    def set_light_power(self, p):
        self._check(_lib.fr_set_light_power(self._ctx, float(p)))

    def set_diffuse_max_depth(self, d):
        self._check(_lib.fr_set_diffuse_max_depth(self._ctx, int(d)))

    def ray_count(self):
        v = C.c_uint32()
        self._check(_lib.fr_ray_count(self._ctx, C.byref(v)))
        return v.value

    def gaze_target(self):
        v = (C.c_float * 3)()
        self._check(_lib.fr_gaze_target(self._ctx, v))
        return np.array(v[:], np.float32)

    def get_texture(self, name):
        return int(name)

    def view(self, buf) -> fr_buffer_view:
        v = fr_buffer_view()
        self._check(_lib.fr_get_buffer(self._ctx, int(buf), C.byref(v)))
        return v

    def read(self, buf) -> np.ndarray:
        v = self.view(buf)
        if v.format == 0:
            out = np.empty((v.height, v.width, 4), np.float32)
        elif v.format == 1:
            out = np.empty((v.width,), np.uint32)
        else:
            out = np.empty((v.height, v.width), np.uint8)
        self._check(_lib.fr_read_buffer(self._ctx, int(buf), out.ctypes.data, out.nbytes))
        return out

    def write(self, buf, arr: np.ndarray):
        arr = np.ascontiguousarray(arr)
        self._check(_lib.fr_write_buffer(self._ctx, int(buf), arr.ctypes.data, arr.nbytes))

    def stats(self) -> dict:
        s = fr_stats()
        self._check(_lib.fr_get_stats(self._ctx, C.byref(s)))
        return {n: (list(getattr(s, n)) if n == "diag" else getattr(s, n)) for n, _ in fr_stats._fields_}

    def reset_stats(self):
        self._check(_lib.fr_reset_stats(self._ctx))

    def kernel_timing(self, enable: bool):
        """Starts (or stops) the live HIP-event timing of entry 3 inside pipelined frames."""
        self._check(_lib.fr_kernel_timing(self._ctx, 1 if enable else 0))

    def kernel_times(self) -> dict:
        """{frames, shading_ms, shade_paths_ms}: stages timed since kernel_timing(True), summed ms."""
        t = fr_stage_times()
        self._check(_lib.fr_kernel_times(self._ctx, C.byref(t)))
        return {"frames": t.frames, "shading_ms": t.shading_ms, "shade_paths_ms": t.shade_paths_ms}

    def frame_clock(self, enable: bool):
        """fr_frame_clock: starts (or stops and clears) the per-frame latency / interval events of fr_frame."""
        self._check(_lib.fr_frame_clock(self._ctx, 1 if enable else 0))

    def frame_clock_read(self, cap=100000):
        """(latency_ms, interval_ms) numpy arrays of every frame since frame_clock(True)."""
        lat = (C.c_float * cap)()
        itv = (C.c_float * cap)()
        nl, ni = C.c_int(0), C.c_int(0)
        self._check(_lib.fr_frame_clock_read(self._ctx, lat, itv, cap, C.byref(nl), C.byref(ni)))
        return (np.frombuffer(lat, np.float32, nl.value).copy(), np.frombuffer(itv, np.float32, ni.value).copy())

    def _frame(self, fn, timing):
        t = fr_frame_timing() if timing else None
        self._check(fn(self._ctx, C.byref(t) if timing else None))
        if not timing:
            return None
        return {n: getattr(t, n) for n, _ in fr_frame_timing._fields_}

    def frame(self, timing=True):
        """One iteration of the FR/main.cpp:253-358 loop body on the device."""
        return self._frame(_lib.fr_frame, timing)

    def set_pipeline_mode(self, mode):
        """fr_set_pipeline_mode: PIPELINE_THROUGHPUT (0, frames enqueued back to back) or PIPELINE_LATENCY (1,
        one trace half in flight: fr_frame waits for the previous frame's path trace before it starts)."""
        self._check(_lib.fr_set_pipeline_mode(self._ctx, int(mode)))

    def set_sample_sum(self, mode):
        """fr_set_sample_sum: 0 fp32, 1 by frame size (default), 2 fixed point with the tail handoff."""
        self._check(_lib.fr_set_sample_sum(self._ctx, int(mode)))

    def shard_unpack_active_enqueue(self, device_ptr, capacity, count):
        """fr_shard_unpack_active without synchronisation (enqueued on the context stream)."""
        self._check(_lib.fr_shard_unpack_active_enqueue(self._ctx, C.c_void_p(device_ptr), int(capacity) * 20,
                                                        int(capacity), int(count)))

    def set_front_local(self, on=True):
        """fr_set_front_local: front stages on this rank's tiles plus halo only (a still camera's tracer)."""
        self._check(_lib.fr_set_front_local(self._ctx, int(bool(on))))

    def set_recon_chains(self, chains):
        """Reconstruction chains this context runs: bit 0 JFA -> Sibson, bit 1 pull-push -> A-Trous."""
        self._check(_lib.fr_set_recon_chains(self._ctx, int(chains)))

    def trace_frame(self, timing=True):
        """The trace half of a frame (update -> entries 0..3)."""
        return self._frame(_lib.fr_trace_frame, timing)

    def reconstruct_frame(self, timing=True):
        """The reconstruction half of a frame (JFA -> Sibson -> pull-push -> A-Trous)."""
        return self._frame(_lib.fr_reconstruct_frame, timing)

    def snapshot(self) -> bytes:
        """fr_snapshot: the temporal state (history / depth pairs, pull-push atlases, frame counter, camera)."""
        n = C.c_size_t()
        self._check(_lib.fr_snapshot_bytes(self._ctx, C.byref(n)))
        buf = (C.c_uint8 * n.value)()
        self._check(_lib.fr_snapshot(self._ctx, buf, n.value))
        return bytes(buf)

    def restore(self, snap: bytes):
        """fr_restore: load a snapshot of a context with the same size, spp and scene."""
        buf = (C.c_uint8 * len(snap)).from_buffer_copy(snap)
        self._check(_lib.fr_restore(self._ctx, buf, len(snap)))

    def copy_buffer(self, buffer_id, device_ptr, nbytes):
        """Device-to-device copy of a buffer into memory the caller owns (e.g. a torch tensor)."""
        self._check(_lib.fr_copy_buffer(self._ctx, int(buffer_id), C.c_void_p(device_ptr), int(nbytes)))

    def composite_views(self, views_ptr, nviews, out_ptr, out_bytes):
        """Side-by-side composite of nviews W x H device images into (nviews W) x H (device pointers)."""
        self._check(_lib.fr_composite_views(self._ctx, C.c_void_p(views_ptr), int(nviews), C.c_void_p(out_ptr),
                                            int(out_bytes)))

    def rebuild_bvh(self) -> float:
        """Re-indexes the current triangles with the GPU builder; returns its wall time in ms."""
        return self._launch(_lib.fr_rebuild_bvh)

    def set_positions(self, xyz: np.ndarray):
        """New world-space vertex positions (ntris x 3 x 3 float32, scene triangle order), then a GPU
        rebuild of the BVH."""
        a = np.ascontiguousarray(xyz, dtype=np.float32)
        n = a.size // 9
        self._check(_lib.fr_set_positions(self._ctx, a.ctypes.data_as(C.POINTER(C.c_float)), n))

    def set_gaze(self, xpos, ypos, fullscreen=False):
        """cursorPosCallback (FR/gui.cpp:48-66): the cursor in window coordinates (y down);
        g_gaze = (LONG(xpos), LONG(ypos * adjust_scale)), adjust_scale 1 in full screen, 1.25 in a window."""
        self._check(_lib.fr_set_gaze(self._ctx, float(xpos), float(ypos), 1 if fullscreen else 0))

    def reset_gaze(self):
        """framebufferSizeCallback (FR/gui.cpp:32-35): g_gaze = (W / 2, H / 2)."""
        self._check(_lib.fr_reset_gaze(self._ctx))

    # tile sharding of one view across ranks (include/fovrt.h, fr_set_shard)
    def set_shard(self, rank, count, tile=128, first_tracer=0):
        """fr_set_shard_ex: tiles dealt round robin over ranks first_tracer .. count-1."""
        self._check(_lib.fr_set_shard_ex(self._ctx, int(rank), int(count), int(tile), int(first_tracer)))

    def set_shard_plan(self, rank, count, tile, owner):
        """fr_set_shard_plan: owner[t] (uint8, one per tile in raster order) traces tile t."""
        o = np.ascontiguousarray(owner, dtype=np.uint8)
        self._check(_lib.fr_set_shard_plan(self._ctx, int(rank), int(count), int(tile),
                                           o.ctypes.data_as(C.POINTER(C.c_uint8)), o.size))

    def shard_counts(self, n) -> np.ndarray:
        """Active pixels of every view rank in the last front stages, from this rank's own full mask."""
        out = np.zeros(int(n), np.uint32)
        self._check(_lib.fr_shard_counts(self._ctx, out.ctypes.data_as(C.POINTER(C.c_uint32)), int(n)))
        return out

    def shard_texels(self) -> int:
        n = C.c_size_t()
        self._check(_lib.fr_shard_texels(self._ctx, C.byref(n)))
        return n.value

    def shard_pack(self, buffer_id, device_ptr, nbytes):
        """Packs this rank's tiles of an RGBA32F buffer into the device slab at device_ptr."""
        self._check(_lib.fr_shard_pack(self._ctx, int(buffer_id), C.c_void_p(device_ptr), int(nbytes)))

    def shard_unpack(self, buffer_id, src_rank, device_ptr, nbytes):
        """Writes rank src_rank's tiles from the device slab at device_ptr into the buffer."""
        self._check(_lib.fr_shard_unpack(self._ctx, int(buffer_id), int(src_rank), C.c_void_p(device_ptr),
                                         int(nbytes)))

    def shard_pack_active(self, device_ptr, capacity, slab_bytes=None) -> int:
        """Packs the pixels this rank's last trace half shaded (capacity x 20 B slab); returns their count."""
        n = C.c_uint32()
        nb = int(capacity) * 20 if slab_bytes is None else int(slab_bytes)
        self._check(_lib.fr_shard_pack_active(self._ctx, C.c_void_p(device_ptr), nb, int(capacity), C.byref(n)))
        return n.value

    def shard_unpack_active(self, device_ptr, capacity, count, slab_bytes=None):
        """Adds this rank's reprojected history to another rank's packed pixels (their radiance) and scatters
        the sums into HISTORY_CACHE and SHADING."""
        nb = int(capacity) * 20 if slab_bytes is None else int(slab_bytes)
        self._check(_lib.fr_shard_unpack_active(self._ctx, C.c_void_p(device_ptr), nb, int(capacity), int(count)))

    def synchronize(self):
        self._check(_lib.fr_synchronize(self._ctx))

    def scene_arrays(self) -> dict:
        a = fr_scene_arrays()
        self._check(_lib.fr_scene_export(self._ctx, C.byref(a)))
        return _arrays_to_dict(a)


def _arrays_to_dict(a: fr_scene_arrays) -> dict:
        n = a.num_tris
        tex = []
        for i in range(a.num_textures):
            w, h = a.tex_dims[2 * i], a.tex_dims[2 * i + 1]
            tex.append(np.ctypeslib.as_array(a.tex_data[i], shape=(h, w, 4)).copy())
        return {
            "pos": np.ctypeslib.as_array(a.pos, shape=(n, 9)).copy(),
            "nrm": np.ctypeslib.as_array(a.nrm, shape=(n, 9)).copy(),
            "uv": np.ctypeslib.as_array(a.uv, shape=(n, 6)).copy(),
            "flags": np.ctypeslib.as_array(a.flags, shape=(n,)).copy(),
            "materials": np.ctypeslib.as_array(a.materials, shape=(a.num_materials, 2)).copy(),
            "textures": tex,
            "envmap": a.envmap,
            "light": np.array(a.light[:], np.float32),
            "bbox": np.array(a.bbox[:], np.float32),
            "bvh_nodes": a.bvh_nodes,
            "bvh_depth": a.bvh_depth,
            "bvh_max_stack": a.bvh_max_stack,
        }


class Scene:
    """Host-only preset scene (fr_scene_create): no device required."""

    def __init__(self, config: Config):
        lib = load_library()
        self._cfg = config.to_c()
        h = C.c_void_p()
        rc = lib.fr_scene_create(C.byref(self._cfg), C.byref(h))
        if rc:
            raise FovrtError(rc, lib.fr_last_error(None).decode())
        self._h = h

    def arrays(self) -> dict:
        a = fr_scene_arrays()
        rc = _lib.fr_scene_get_arrays(self._h, C.byref(a))
        if rc:
            raise FovrtError(rc, "fr_scene_get_arrays")
        return _arrays_to_dict(a)

    def __del__(self):
        if getattr(self, "_h", None) is not None and _lib is not None:
            _lib.fr_scene_destroy(self._h)
            self._h = None


class _Pass:
    def __init__(self, tracer: PathTracer):
        self.tracer = tracer

    def resetShader(self):  # GLSL reload (FR/JumpFlooding.cpp:51-58): nothing to reload here
        pass


class JumpFlooding(_Pass):
    """JumpFlooding::render(rt, query, elapsed, done) (FR/JumpFlooding.cpp:60-140)."""
    coordTex = TextureName.JFA_COORD
    colorTex = TextureName.JFA_COLOR

    def render(self, rt=TextureName.SHADING):
        ns = C.c_uint64()
        self.tracer._check(_lib.fr_jfa_render(self.tracer._ctx, int(rt), C.byref(ns)))
        return ns.value


class LogPolarTransform(_Pass):
    """LogPolarTransform::render(pt, query, elapsed, done) (FR/Log_Polar_Transform.cpp:40-106)."""
    logPolarTex = TextureName.LOGPOLAR
    ilogPolarTex = TextureName.LOGPOLAR_INVERSE

    def render(self, pt=TextureName.PULLPUSH):
        ns = C.c_uint64()
        self.tracer._check(_lib.fr_logpolar_render(self.tracer._ctx, int(pt), C.byref(ns)))
        return ns.value


class SibsonInterpolation(_Pass):
    """SibsonInterpolation::render(coord, color, ...) (FR/SibsonInterpolation.cpp:28-53)."""
    outputTex = TextureName.SIBSON

    def render(self, coord=TextureName.JFA_COORD, color=TextureName.JFA_COLOR):
        if coord != TextureName.JFA_COORD or color != TextureName.JFA_COLOR:
            raise FovrtError(FR_E_UNSUPPORTED, "Sibson reads the JumpFlooding outputs")
        ns = C.c_uint64()
        self.tracer._check(_lib.fr_sibson_render(self.tracer._ctx, C.byref(ns)))
        return ns.value


class PullPushInterpolation(_Pass):
    """PullPushInterpolation::render(sparse, ...) (FR/PullPushInterpolation.cpp:48-238)."""
    outputTex = TextureName.PULLPUSH

    def render(self, sparse=TextureName.SHADING):
        ns = C.c_uint64()
        self.tracer._check(_lib.fr_pullpush_render(self.tracer._ctx, int(sparse), C.byref(ns)))
        return ns.value


class ATrous(_Pass):
    """ATrous::render(count, pos, nrm, col, rt, frame, ...) (FR/ATrous.cpp:47-132)."""
    colorTex = TextureName.ATROUS

    def render(self, count=1, positionTex=TextureName.POSITION, normalTex=TextureName.NORMAL,
               colorTex=TextureName.PULLPUSH, rtTex=None, frame=0):
        ns = C.c_uint64()
        self.tracer._check(_lib.fr_atrous_render(self.tracer._ctx, int(count), int(positionTex), int(normalTex),
                                                 int(colorTex), C.byref(ns)))
        return ns.value


def version():
    return load_library().fr_version().decode()


def shard_plan(width, height, tile, count, weights=None) -> np.ndarray:
    """fr_shard_plan (host only): tile owners dealt by smooth weighted round robin in raster order."""
    lib = load_library()
    nt = ((width + tile - 1) // tile) * ((height + tile - 1) // tile)
    owner = np.zeros(nt, np.uint8)
    w = None if weights is None else (C.c_float * count)(*[float(x) for x in weights])
    rc = lib.fr_shard_plan(int(width), int(height), int(tile), int(count), w,
                           owner.ctypes.data_as(C.POINTER(C.c_uint8)), nt)
    if rc:
        raise FovrtError(rc, lib.fr_last_error(None).decode())
    return owner


def group_plan(width, height, ranks_per_view, tile=128, split_recon=True, recon_cost=None, weights=None,
               jfa_ranks=0) -> np.ndarray:
    """fr_group_plan (host only): the tile plan fr_group_create deals for one view (view rank per tile)."""
    lib = load_library()
    cfg = fr_group_config()
    lib.fr_group_config_default(C.byref(cfg))
    cfg.tile, cfg.split_recon, cfg.jfa_ranks = int(tile), int(bool(split_recon)), int(jfa_ranks)
    if recon_cost is not None:
        cfg.recon_cost[0], cfg.recon_cost[1] = float(recon_cost[0]), float(recon_cost[1])
    if weights is not None:
        for i, w in enumerate(weights):
            cfg.weights[i] = float(w)
    nt = ((width + tile - 1) // tile) * ((height + tile - 1) // tile)
    owner = np.zeros(nt, np.uint8)
    rc = lib.fr_group_plan(int(width), int(height), int(ranks_per_view), C.byref(cfg), owner.ctypes.data, nt)
    if rc:
        raise FovrtError(rc, lib.fr_group_last_error().decode())
    return owner


def rccl_unique_id() -> bytes:
    """fr_rccl_unique_id: the 128-byte RCCL id rank 0 creates and every rank passes to Group.rccl."""
    lib = load_library()
    buf = (C.c_uint8 * 128)()
    rc = lib.fr_rccl_unique_id(buf)
    if rc:
        raise FovrtError(rc, lib.fr_group_last_error().decode())
    return bytes(buf)


class Group:
    """fr_group_*: R ranks (one PathTracer each) rendering `views` views, tile-sharded, with the sparse
    gather to the reconstruction ranks and the optional composite on rank 0 (include/fovrt.h).

    Group(tracers) puts every rank in this process (device-to-device copies); Group.rccl(tracer, id,
    nranks, rank) makes this process's tracer one rank of an RCCL communicator."""

    def __init__(self, tracers, views=1, tile=128, split_recon=True, moving_camera=False, composite=False,
                 recon_cost=None, weights=None, sample_sum=None, front_local=None, jfa_ranks=None,
                 _comm=None):
        lib = load_library()
        cfg = fr_group_config()
        lib.fr_group_config_default(C.byref(cfg))
        cfg.views, cfg.tile = int(views), int(tile)
        cfg.split_recon, cfg.moving_camera, cfg.composite = int(bool(split_recon)), int(bool(moving_camera)), int(bool(composite))
        if recon_cost is not None:
            cfg.recon_cost[0], cfg.recon_cost[1] = float(recon_cost[0]), float(recon_cost[1])
        if weights is not None:
            for i, w in enumerate(weights):
                cfg.weights[i] = float(w)
        if sample_sum is not None:
            cfg.sample_sum = int(sample_sum)
        if front_local is not None:
            cfg.front_local = int(bool(front_local))
        if jfa_ranks is not None:
            cfg.jfa_ranks = int(jfa_ranks)
        self.tracers = list(tracers)
        arr = (C.c_void_p * len(self.tracers))(*[t._ctx.value for t in self.tracers])
        h = C.c_void_p()
        rc = lib.fr_group_create(arr, len(self.tracers), _comm, C.byref(cfg), C.byref(h))
        if rc:
            raise FovrtError(rc, lib.fr_group_last_error().decode())
        self._h = h
        self._comm = _comm
        self._owns_comm = False
        self.config = cfg
        for t in self.tracers:
            if not hasattr(t, "_groups"):
                t._groups = []
            t._groups.append(self)

    @classmethod
    def rccl(cls, tracer, unique_id: bytes, nranks, rank, **kw):
        lib = load_library()
        buf = (C.c_uint8 * 128).from_buffer_copy(unique_id)
        comm = C.c_void_p()
        rc = lib.fr_rccl_comm_init(buf, int(nranks), int(rank), int(tracer.config.device), C.byref(comm))
        if rc:
            raise FovrtError(rc, lib.fr_group_last_error().decode())
        try:
            g = cls([tracer], _comm=comm, **kw)
        except Exception:
            lib.fr_rccl_comm_destroy(comm)
            raise
        g._owns_comm = True
        return g

    def _check(self, rc):
        if rc:
            raise FovrtError(rc, _lib.fr_group_last_error().decode())

    def frame(self, timing=False):
        """One frame of every local rank; timing=True returns one stage-time dict per local rank."""
        if not timing:
            self._check(_lib.fr_group_frame(self._h, None))
            return None
        t = (fr_frame_timing * len(self.tracers))()
        self._check(_lib.fr_group_frame(self._h, t))
        return [{n: getattr(x, n) for n, _ in fr_frame_timing._fields_} for x in t]

    def composite(self, device_ptr, nbytes):
        self._check(_lib.fr_group_composite(self._h, C.c_void_p(device_ptr), int(nbytes)))

    def rank_info(self, i):
        v, vr, ch, tl = C.c_int(), C.c_int(), C.c_int(), C.c_int()
        self._check(_lib.fr_group_rank_info(self._h, int(i), C.byref(v), C.byref(vr), C.byref(ch), C.byref(tl)))
        return {"view": v.value, "view_rank": vr.value, "chains": ch.value, "tiles": tl.value}

    def output_ranks(self, view=0):
        """fr_group_output_ranks: (rank holding the last frame's JFA / Sibson, rank holding its A-Trous)."""
        a, b = C.c_int(), C.c_int()
        self._check(_lib.fr_group_output_ranks(self._h, int(view), C.byref(a), C.byref(b)))
        return a.value, b.value

    def tile_owners(self, width, height):
        """fr_group_tile_owners: the view rank tracing each screen tile, as a (tiles_y, tiles_x) array."""
        T = int(self.config.tile)
        tx, ty = (width + T - 1) // T, (height + T - 1) // T
        out = np.zeros(tx * ty, np.uint8)
        self._check(_lib.fr_group_tile_owners(self._h, out.ctypes.data, out.size))
        return out.reshape(ty, tx)

    def synchronize(self):
        self._check(_lib.fr_group_synchronize(self._h))

    def destroy(self):
        if getattr(self, "_h", None) is not None and _lib is not None:
            _lib.fr_group_destroy(self._h)
            self._h = None
            if self._owns_comm and self._comm is not None:
                _lib.fr_rccl_comm_destroy(self._comm)
                self._comm = None
        # break the tracer <-> group reference cycle: after an explicit destroy both sides are freed by
        # reference counting again (their GPU memory no longer waits for the cycle collector)
        for t in getattr(self, "tracers", ()):
            gs = getattr(t, "_groups", None)
            if gs is not None and self in gs:
                gs.remove(self)
        self.tracers = []

    def __del__(self):
        self.destroy()
