"""ctypes binding of libg2048.so (the C ABI in include/g2048.h).

The library is built in-tree by __graft_entry__.build() (hipcc --offload-arch=gfx950).  There is
no CPU fallback: if the library is missing or no GPU is visible, every entry point raises.
torch is imported first so that libg2048.so binds to the same HIP runtime instance as torch
(both carry SONAME libamdhip64.so.7); device buffers are torch tensors passed by pointer.
"""
from __future__ import annotations

import ctypes as C
import os

import torch  # noqa: F401  (must be loaded before the HIP library, see module docstring)

LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libg2048.so")

G2048_OK, G2048_EINVAL, G2048_EHIP, G2048_ENOMEM, G2048_EBADINPUT = 0, -1, -2, -3, -4
P4_10, EGREEDY_FIXED, NO_AUTORESET = 1, 2, 4
F32, F64 = 0, 1
ASTAR_SPAWN_PHILOX, ASTAR_SPAWN_FIRST_EMPTY = 0, 1
ABI_VERSION = 5  # include/g2048.h G2048_ABI_VERSION
MAX_BOARDS = (1 << 31) - 256  # include/g2048.h G2048_MAX_BOARDS
REPLAY_SECTION_PAD = 4352  # include/g2048.h G2048_REPLAY_SECTION_PAD

# every symbol include/g2048.h declares, with (restype, argtypes)
_vp, _i64, _u64, _i32, _u32, _int, _dbl = (C.c_void_p, C.c_int64, C.c_uint64, C.c_int32,
                                          C.c_uint32, C.c_int, C.c_double)
_pp = C.POINTER(C.c_void_p)
SIGNATURES = {
    "g2048_env_create": (_int, [_pp, _i64, _u64, _u64, _int, _u32, _vp]),
    "g2048_env_wrap": (_int, [_pp, _i64, _u64, _u64, _int, _u32, _vp, _vp, _vp, _vp, _int, _vp]),
    "g2048_env_destroy": (None, [_vp]),
    "g2048_env_views": (_int, [_vp, _pp, _pp, _pp, _pp]),
    "g2048_env_size": (_i64, [_vp]),
    "g2048_env_reset": (_int, [_vp, _vp, _vp]),
    "g2048_env_step": (_int, [_vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    "g2048_env_step_egreedy": (_int, [_vp, _vp, _int, _vp, _dbl, _vp, _vp, _vp, _vp, _vp]),
    "g2048_env_step_egreedy_schedule": (_int, [_vp, _vp, _int, _dbl, _dbl, _vp, _vp, _vp, _vp,
                                               _vp]),
    "g2048_env_step_inject": (_int, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    "g2048_env_rollout": (_int, [_vp, _i32, _vp, _vp, _vp]),
    "g2048_env_error_count": (_int, [_vp, C.POINTER(C.c_int64), _vp]),
    "g2048_env_get_epoch": (_int, [_vp, C.POINTER(C.c_uint32)]),
    "g2048_env_set_epoch": (_int, [_vp, _u32]),
    "g2048_env_set_episode_log": (_int, [_vp, _vp, _i64, _vp]),
    "g2048_env_legal_mask": (_int, [_vp, _vp, _vp]),
    "g2048_env_score_moves": (_int, [_vp, _vp, _vp]),
    "g2048_env_step_egreedy_dense64": (_int, [_vp, _vp, _vp, _dbl, _dbl, _dbl, _vp, _vp, _vp, _vp,
                                              _vp, _vp]),
    "g2048_env_step_egreedy_dense64_f64": (_int, [_vp, _vp, _vp, _dbl, _dbl, _dbl, _vp, _vp, _vp, _vp,
                                              _vp, _vp]),
    "g2048_replay_create": (_int, [_pp, _i64, _int, _vp]),
    "g2048_replay_wrap": (_int, [_pp, _i64, _int, _vp, _vp, _vp, _vp, _vp, _vp]),
    "g2048_replay_destroy": (None, [_vp]),
    "g2048_replay_views": (_int, [_vp, _pp, _pp, _pp, _pp, _pp, _pp]),
    "g2048_replay_sample_encode": (_int, [_vp, _vp, _i64, _u64, _u64, _int, _vp, _vp, _vp, _vp,
                                          _vp, _vp, _vp]),
    "g2048_convnet_forward": (_int, [_vp, _vp, _vp, _i64, _vp, _vp]),
    "g2048_convnet_forward_greedy": (_int, [_vp, _vp, _vp, _dbl, _dbl, _dbl, _vp, _vp]),
    "g2048_convnet_train_workspace": (_i64, [_i64]),
    "g2048_convnet_train_grad": (_int, [_vp, _vp, _vp, _vp, _vp, _i64, _vp, _vp, _vp, _vp, _vp]),
    "g2048_convnet_train_adam": (_int, [_vp, _vp, _vp, _vp, _vp, _i64, _vp, _vp, _vp, _vp, _vp,
                                        _vp, _dbl, _dbl, _dbl, _dbl, _vp, _u64, _vp]),
    "g2048_convnet_targets": (_int, [_vp, _vp, _vp, _vp, _i64, _u64, _vp, C.c_float, _int, _vp,
                                     _vp, _vp]),
    "g2048_adam_step": (_int, [_vp, _vp, _int, _vp, _vp, _vp, _vp, _dbl, _dbl, _dbl, _dbl, _vp]),
    "g2048_adam_step_sync": (_int, [_vp, _vp, _int, _vp, _vp, _vp, _vp, _dbl, _dbl, _dbl, _dbl,
                                    _vp, _u64, _vp]),
    "g2048_dense64_forward": (_int, [_vp, _vp, _vp, _i64, _vp, _vp]),
    "g2048_dense64_targets": (_int, [_vp, _vp, _vp, _vp, _i64, _u64, _vp, C.c_float, _int, _vp,
                                     _vp, _vp]),
    "g2048_dense64_train_workspace": (_i64, [_i64]),
    "g2048_dense64_train_grad": (_int, [_vp, _vp, _vp, _vp, _vp, _i64, _vp, _vp, _vp, _vp, _vp]),
    "g2048_dense64_update_workspace": (_i64, [_i64]),
    "g2048_dense64_update": (_int, [_vp, _vp, _vp, _vp, _i64, _u64, _vp, C.c_float, _int, _vp, _vp, _vp,
                                    _vp, _vp, _vp, _vp, _dbl, _dbl, _dbl, _dbl, _u64, _vp]),
    "g2048_dense64_update_f64_workspace": (_i64, [_i64]),
    "g2048_dense64_update_f64": (_int, [_vp, _vp, _vp, _vp, _i64, _u64, _vp, C.c_float, _int, _vp,
                                        _vp, _vp, _vp, _vp, _vp, _vp, _dbl, _dbl, _dbl, _dbl,
                                        _u64, _vp]),
    "g2048_adam_step_sync_f64": (_int, [_vp, _vp, _int, _vp, _vp, _vp, _vp, _dbl, _dbl, _dbl, _dbl,
                                        _vp, _u64, _vp]),
    "g2048_densenet_update_workspace": (_i64, [_i64, _int]),
    "g2048_densenet_update": (_int, [_vp, _vp, _int, _vp, _vp, _i64, _u64, _vp, C.c_float, _int,
                                     _vp, _vp, _vp, _vp, _vp, _vp, _vp, _dbl, _dbl, _dbl, _dbl,
                                     _u64, _vp]),
    "g2048_adam_step_scaled": (_int, [_vp, _vp, _int, _vp, _vp, _vp, _vp, _dbl, _dbl, _dbl, _dbl,
                                      _vp, _u64, _dbl, _vp]),
    "g2048_adam_step_scaled_f64": (_int, [_vp, _vp, _int, _vp, _vp, _vp, _vp, _dbl, _dbl, _dbl,
                                          _dbl, _vp, _u64, _dbl, _vp]),
    "g2048_convnet_update_f64_workspace": (_i64, [_i64]),
    "g2048_convnet_pack_f64": (_int, [_vp, _vp, _vp, _vp]),
    "g2048_convnet_forward_f64": (_int, [_vp, _vp, _vp, _i64, _vp, _vp, _vp]),
    "g2048_convnet_forward_greedy_f64": (_int, [_vp, _vp, _vp, _dbl, _dbl, _dbl, _vp, _vp, _vp]),
    "g2048_convnet_update_f64": (_int, [_vp, _vp, _vp, _vp, _i64, _u64, _vp, C.c_float, _int, _vp,
                                        _vp, _vp, _vp, _vp, _vp, _vp, _dbl, _dbl, _dbl, _dbl,
                                        _u64, _vp]),
    "g2048_convnet_update": (_int, [_vp, _vp, _vp, _vp, _i64, _u64, _vp, C.c_float, _int, _vp, _vp, _vp,
                                    _vp, _vp, _vp, _vp, _dbl, _dbl, _dbl, _dbl, _u64, _vp]),
    "g2048_densenet_forward": (_int, [_vp, _int, _vp, _vp, _i64, _vp, _vp]),
    "g2048_densenet_forward_greedy": (_int, [_vp, _int, _vp, _vp, _dbl, _dbl, _dbl, _vp, _vp]),
    "g2048_astar_search": (_int, [_vp, _i64, _int, _u64, _u64, _int, _i64, _i64, _vp, _vp, _vp,
                                  _vp, _vp, _vp, _vp]),
    "g2048_last_error": (C.c_char_p, []),
    "g2048_abi_version": (_int, []),
}



class ConvNetParams(C.Structure):
    """g2048_convnet_params / g2048_convnet_params_f64: device pointers of the conv Q-net's 8
    tensors (fp32 / fp64)."""
    _fields_ = [(n, C.c_void_p) for n in ("w1", "b1", "w2", "b2", "fc1_w", "fc1_b", "fc2_w",
                                          "fc2_b")]




class DenseNetParams(C.Structure):
    """g2048_densenet_params: device pointers of the reference dense Q-net's 8 tensors."""
    _fields_ = [(n, C.c_void_p) for n in ("w1", "b1", "w2", "b2", "w3", "b3", "w4", "b4")]


class Dense64Params(C.Structure):
    """g2048_dense64_params / g2048_dense64_params_f64: device pointers of the dense 16-64-4
    Q-net's 4 tensors (fp32 / fp64)."""
    _fields_ = [(n, C.c_void_p) for n in ("w1", "b1", "w2", "b2")]


_lib = None


class NativeError(RuntimeError):
    pass


def load() -> C.CDLL:
    """Load libg2048.so and bind every declared symbol (no GPU needed for this)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} is not built: run `python -c 'import __graft_entry__ as g; "
                              "g.build()'` (hipcc --offload-arch=gfx950)")
        lib = C.CDLL(LIB_PATH, mode=C.RTLD_GLOBAL)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        if lib.g2048_abi_version() != ABI_VERSION:
            raise ImportError("libg2048.so ABI version mismatch")
        _lib = lib
    return _lib


def check(rc: int, what: str = "") -> None:
    if rc != G2048_OK:
        msg = load().g2048_last_error().decode(errors="replace")
        raise NativeError(f"{what or 'g2048'} failed ({rc}): {msg}")


def ptr(t) -> int | None:
    return None if t is None else t.data_ptr()


def stream_of(device: torch.device) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def require_gpu(device) -> torch.device:
    dev = torch.device(device)
    if dev.type != "cuda":
        raise NativeError(f"g2048 runs on the GPU only (got device {dev}); there is no CPU path")
    if not torch.cuda.is_available():
        raise NativeError("g2048 needs a visible MI355X GPU (torch.cuda.is_available() is False)")
    if dev.index is None:
        dev = torch.device("cuda", torch.cuda.current_device())
    return dev
