"""ctypes binding of ``libmtsac.so`` (the C-ABI declared in ``include/mtsac.h``).

This is the reference-side binding a maintainer would add.
There is no fallback: if the HIP library is missing or fails to load, every
product entry point raises :class:`MTSACLibraryError`.
"""

from __future__ import annotations

import ctypes
import os
import pathlib

_HERE = pathlib.Path(__file__).resolve().parent
LIB_PATH = pathlib.Path(os.environ.get("MTSAC_LIB", _HERE / "libmtsac.so"))

NUM_LOGS = 10
# enum mtsac_precision (include/mtsac.h)
FP32, FP32_SPLIT3, BF16, FP32_SPLIT2H = 0, 1, 2, 3
PRECISIONS = {"fp32": FP32, "split3": FP32_SPLIT3, "bf16": BF16, "split2h": FP32_SPLIT2H}
LOG_KEYS = (
    "losses/qf_values",
    "losses/qf_loss",
    "metrics/critic_grad_magnitude",
    "metrics/critic_params_norm",
    "losses/actor_loss",
    "metrics/actor_grad_magnitude",
    "metrics/actor_params_norm",
    "metrics/explore_loss",
    "losses/alpha_loss",
    "alpha",
)

# enum mtsac_tensor
ACTOR, CRITIC, CRITIC_TARGET, LOG_ALPHA = 0, 1, 2, 3
ACTOR_ADAM_MU, ACTOR_ADAM_NU, CRITIC_ADAM_MU, CRITIC_ADAM_NU, ALPHA_ADAM_MU, ALPHA_ADAM_NU = 4, 5, 6, 7, 8, 9


class MTSACLibraryError(RuntimeError):
    pass


class MTSACError(RuntimeError):
    pass


class Config(ctypes.Structure):
    _fields_ = [
        ("num_tasks", ctypes.c_int32),
        ("task_begin", ctypes.c_int32),
        ("task_count", ctypes.c_int32),
        ("obs_dim", ctypes.c_int32),
        ("action_dim", ctypes.c_int32),
        ("actor_width", ctypes.c_int32),
        ("actor_depth", ctypes.c_int32),
        ("critic_width", ctypes.c_int32),
        ("critic_depth", ctypes.c_int32),
        ("num_critics", ctypes.c_int32),
        ("batch_per_task", ctypes.c_int32),
        ("capacity", ctypes.c_int64),
        ("gamma", ctypes.c_float),
        ("tau", ctypes.c_float),
        ("actor_lr", ctypes.c_float),
        ("critic_lr", ctypes.c_float),
        ("alpha_lr", ctypes.c_float),
        ("actor_max_grad_norm", ctypes.c_float),
        ("critic_max_grad_norm", ctypes.c_float),
        ("alpha_max_grad_norm", ctypes.c_float),
        ("adam_b1", ctypes.c_float),
        ("adam_b2", ctypes.c_float),
        ("adam_eps", ctypes.c_float),
        ("initial_temperature", ctypes.c_float),
        ("log_std_min", ctypes.c_float),
        ("log_std_max", ctypes.c_float),
        ("clip", ctypes.c_int32),
        ("use_task_weights", ctypes.c_int32),
        ("normalize_rewards", ctypes.c_int32),
        ("precision", ctypes.c_int32),
        ("noise_seed", ctypes.c_uint64),
    ]


class Batch(ctypes.Structure):
    _fields_ = [
        ("observations", ctypes.c_void_p),
        ("actions", ctypes.c_void_p),
        ("next_observations", ctypes.c_void_p),
        ("dones", ctypes.c_void_p),
        ("rewards", ctypes.c_void_p),
    ]


P = ctypes.c_void_p
I32, I64, U32, U64 = ctypes.c_int32, ctypes.c_int64, ctypes.c_uint32, ctypes.c_uint64
PI32, PI64, PU32, PU64 = (ctypes.POINTER(t) for t in (I32, I64, U32, U64))
PD = ctypes.POINTER(ctypes.c_double)

# name -> (restype, argtypes); every symbol declared in include/mtsac.h and include/mtsac_debug.h
SIGNATURES = {
    "mtsac_last_error": (ctypes.c_char_p, []),
    "mtsac_abi_version": (ctypes.c_int, []),
    "mtsac_build_stamp": (ctypes.c_char_p, []),
    "mtsac_default_config": (None, [ctypes.POINTER(Config), I32]),
    "mtsac_create": (ctypes.c_int, [ctypes.POINTER(Config), ctypes.c_int, ctypes.POINTER(P)]),
    "mtsac_destroy": (None, [P]),
    "mtsac_param_count": (I64, [P, ctypes.c_int]),
    "mtsac_set_params": (ctypes.c_int, [P, ctypes.c_int, P, I64]),
    "mtsac_get_params": (ctypes.c_int, [P, ctypes.c_int, P, I64]),
    "mtsac_set_adam_count": (ctypes.c_int, [P, ctypes.c_int, I32]),
    "mtsac_get_adam_count": (ctypes.c_int, [P, ctypes.c_int, PI32]),
    "mtsac_buffer_add": (ctypes.c_int, [P, P, P, P, P, P]),
    "mtsac_buffer_add_stream": (ctypes.c_int, [P, P, P, P, P, P, P]),
    "mtsac_buffer_write": (ctypes.c_int, [P, I64, I64, P, P, P, P, P]),
    "mtsac_buffer_read": (ctypes.c_int, [P, I64, I64, P, P, P, P, P]),
    "mtsac_buffer_fill_synthetic": (ctypes.c_int, [P, U64]),
    "mtsac_buffer_set_state": (ctypes.c_int, [P, I64, I32]),
    "mtsac_buffer_get_state": (ctypes.c_int, [P, PI64, PI32]),
    "mtsac_buffer_set_reward_stats": (ctypes.c_int, [P, PD, PD]),
    "mtsac_buffer_get_reward_stats": (ctypes.c_int, [P, PD, PD]),
    "mtsac_rng_set": (ctypes.c_int, [P, U64, U64, U64, U64, I32, U32]),
    "mtsac_rng_get": (ctypes.c_int, [P, PU64, PU64, PU64, PU64, PI32, PU32]),
    "mtsac_sample": (ctypes.c_int, [P, P, P, P, P, P, P]),
    "mtsac_update": (ctypes.c_int, [P, ctypes.POINTER(Batch), P, P]),
    "mtsac_update_many": (ctypes.c_int, [P, I32]),
    "mtsac_get_logs": (ctypes.c_int, [P, P]),
    "mtsac_enable_graph": (ctypes.c_int, [P, I32]),
    "mtsac_synchronize": (ctypes.c_int, [P]),
    "mtsac_eval_action": (ctypes.c_int, [P, P, I32, P]),
    "mtsac_sample_action": (ctypes.c_int, [P, P, I32, P, P]),
    "mtsac_comm_unique_id_size": (ctypes.c_int, []),
    "mtsac_comm_get_unique_id": (ctypes.c_int, [P]),
    "mtsac_comm_init": (ctypes.c_int, [P, P, I32, I32]),
    "mtsac_comm_init_timeout": (ctypes.c_int, [P, P, I32, I32, ctypes.c_double]),
    "mtsac_comm_nranks": (ctypes.c_int, [P, P]),
    "mtsac_get_noise_state": (ctypes.c_int, [P, P, P]),
    "mtsac_set_noise_state": (ctypes.c_int, [P, ctypes.c_uint64, ctypes.c_uint64]),
    "mtsac_set_allreduce_hook": (ctypes.c_int, [P, ctypes.c_void_p, P]),
    "mtsac_set_collective_hook": (ctypes.c_int, [P, ctypes.c_void_p, P, ctypes.c_int32, ctypes.c_int32]),
    "mtsac_set_sharded_optimizer": (ctypes.c_int, [P, ctypes.c_int32]),
    "mtsac_memcpy": (ctypes.c_int, [P, P, I64]),
    "mtsac_set_timing": (ctypes.c_int, [P, I32]),
    "mtsac_get_timing": (ctypes.c_int, [P, I32, PD, PI32, PD]),
    "mtsac_get_timing_kernel": (ctypes.c_int, [P, I32, P, I32]),
    "mtsac_task_gradients": (ctypes.c_int, [P, ctypes.POINTER(Batch), P, P]),
    "mtsac_task_gradient_size": (I64, [P, ctypes.c_int]),
    "mtsac_get_task_gradients": (ctypes.c_int, [P, ctypes.c_int, P, I64]),
    "mtsac_set_task_gradients": (ctypes.c_int, [P, ctypes.c_int, P, I64]),
    "mtsac_task_gradient_select": (ctypes.c_int, [P, ctypes.c_int, P, P]),
    "mtsac_task_gradient_stats": (ctypes.c_int, [P, ctypes.c_int, P, ctypes.c_float, ctypes.c_float, P, P, P, P]),
    "mtsac_debug_gemm_bench": (ctypes.c_int, [ctypes.c_int] * 8 + [PD]),
    "mtsac_debug_gemm_x3p": (ctypes.c_int, [ctypes.c_int] * 4 + [P, ctypes.c_int, P, ctypes.c_int, P, P, P, P]),
    "mtsac_debug_gemm_x3p_bench": (ctypes.c_int, [ctypes.c_int] * 6 + [PD]),
    "mtsac_debug_x3p_geo": (ctypes.c_int, [ctypes.c_int]),
    "mtsac_debug_gemm_x3f": (ctypes.c_int, [ctypes.c_int] * 5 + [P] * 6),
    "mtsac_debug_gemm_fwd_bench": (ctypes.c_int, [ctypes.c_int] * 7 + [PD]),
    "mtsac_debug_x3s_ti": (ctypes.c_int, [ctypes.c_int] * 3),
    "mtsac_debug_drq_groups": (ctypes.c_int, [ctypes.c_int] * 2),
    "mtsac_debug_drq_mfma": (ctypes.c_int, [ctypes.c_int]),
    "mtsac_debug_drq_legacy": (ctypes.c_int, [ctypes.c_int]),
    "mtsac_debug_drq_wgrad_blocks": (ctypes.c_int, [ctypes.c_int]),
    "mtsac_debug_drq_conv_bench": (ctypes.c_int, [ctypes.c_int] * 7 + [ctypes.POINTER(ctypes.c_double)]),
    "mtsac_debug_set_pipeline": (ctypes.c_int, [P, I32]),
    "mtsac_debug_lane_mode": (ctypes.c_int, [P]),
    "mtsac_debug_check_guards": (ctypes.c_int, [P]),
    "mtsac_debug_snapshot": (ctypes.c_int, [P, ctypes.c_int32]),
    "mtsac_debug_read": (ctypes.c_int, [P, ctypes.c_int32, P, ctypes.c_int64]),
    "mtsac_debug_head_selfcheck": (ctypes.c_int, [P]),
    "mtsac_debug_set_bfrag": (ctypes.c_int, [ctypes.c_int32]),
    "mtsac_debug_bfrag": (ctypes.c_int, [P]),
    "mtsac_debug_force_one_stream": (ctypes.c_int, [P, ctypes.c_int32]),
    "mtsac_debug_set_collective_model": (ctypes.c_int, [P, ctypes.c_int32, ctypes.c_double, ctypes.c_int32]),
    "mtsac_debug_timed_launch": (ctypes.c_int, [P, I32, PI32, PD]),
    "mtsac_debug_gemm": (
        ctypes.c_int,
        # precision, kind, epi, batch, M, N, K, A, lda, a_shared, B, ldb, C, ldc, bias, mask, ldm, db
        [ctypes.c_int] * 7 + [P, ctypes.c_int, ctypes.c_int, P, ctypes.c_int, P, ctypes.c_int, P, P, ctypes.c_int, P],
    ),
}


class DrqConfig(ctypes.Structure):  # include/drq.h
    _fields_ = [(n, ctypes.c_int32) for n in ("num_tasks", "n_actions", "n_atoms", "in_ch", "hw", "scale",
                                              "embed_dim", "n_hidden", "batch", "nstep")] + \
               [(n, ctypes.c_float) for n in ("gamma", "v_min", "v_max", "tau", "lr", "b1", "b2", "eps",
                                              "weight_decay", "ln_eps")] + \
               [("capacity", ctypes.c_int64), ("normalize_rewards", ctypes.c_int32), ("buffer_kind", ctypes.c_int32)]


class DrqBatch(ctypes.Structure):
    _fields_ = [(n, ctypes.c_void_p) for n in ("obs", "actions", "next_obs", "dones", "rewards", "task_ids",
                                               "crop_obs", "noise_obs", "crop_next", "noise_next")]


DRQ_PARAMS, DRQ_TARGET, DRQ_ADAM_MU, DRQ_ADAM_NU, DRQ_GRAD = 0, 1, 2, 3, 4
DRQ_NUM_LOGS = 4
DRQ_LOG_KEYS = ("losses/online_logits", "metrics/critic_grad_magnitude", "metrics/critic_params_norm",
                "losses/critic_loss")
SIGNATURES.update({
    "drq_last_error": (ctypes.c_char_p, []),
    "drq_create": (ctypes.c_int, [ctypes.POINTER(DrqConfig), ctypes.c_int, ctypes.POINTER(P)]),
    "drq_destroy": (None, [P]),
    "drq_num_params": (I64, [P]),
    "drq_set_params": (ctypes.c_int, [P, ctypes.c_int, P, I64]),
    "drq_get_params": (ctypes.c_int, [P, ctypes.c_int, P, I64]),
    "drq_set_step": (ctypes.c_int, [P, ctypes.c_int]),
    "drq_get_step": (ctypes.c_int, [P, P]),
    "drq_update": (ctypes.c_int, [P, ctypes.POINTER(DrqBatch)]),
    "drq_update_resident": (ctypes.c_int, [P, ctypes.c_int]),
    "drq_get_logs": (ctypes.c_int, [P, P]),
    "drq_q_values": (ctypes.c_int, [P, P, P, P, P, ctypes.c_int, P]),
    "drq_buffer_add": (ctypes.c_int, [P, P, P, P, P, P, P]),
    "drq_buffer_state": (ctypes.c_int, [P, PI64, PI32]),
    "drq_rng_set": (ctypes.c_int, [P, U64, U64, U64, U64, ctypes.c_int, U32]),
    "drq_sample": (ctypes.c_int, [P]),
    "drq_sample_update": (ctypes.c_int, [P, ctypes.c_int]),
    "drq_sample_rows": (ctypes.c_int, [P, P, P]),
    "drq_sample_rows_update": (ctypes.c_int, [P, P, P, ctypes.c_int]),
    "drq_rng_get": (ctypes.c_int, [P, P]),
    "drq_seed_augment": (ctypes.c_int, [P, ctypes.c_uint64]),
    "drq_task_gradient": (ctypes.c_int, [P, ctypes.POINTER(DrqBatch), ctypes.c_int, ctypes.c_int]),
    "drq_get_task_gradient": (ctypes.c_int, [P, ctypes.c_int, P, I64]),
    "drq_project_task_gradients": (ctypes.c_int, [P, ctypes.c_int, ctypes.c_int, I64, ctypes.c_int, P]),
    "drq_set_timing": (ctypes.c_int, [P, ctypes.c_int]),
    "drq_timing": (ctypes.c_int, [P, P, P, P]),
    "drq_read_batch": (ctypes.c_int, [P, P, P, P, P, P, P, P]),
    "drq_synchronize": (ctypes.c_int, [P]),
})

def source_stamp() -> str | None:
    """sha256 (first 16 hex digits) of the engine sources as mtrl_amd/csrc/Makefile stamps them into the
    library: csrc/*.hip, *.cpp, *.h and include/*.h in sorted path order (as make's $(sort) orders
    the relative paths), concatenated; None when the sources are not in the tree."""
    import hashlib

    csrc = pathlib.Path(__file__).resolve().parent / "csrc"
    if not csrc.is_dir():
        return None
    rel = [f.name for pat in ("*.hip", "*.cpp", "*.h") for f in csrc.glob(pat)]
    rel += ["../../include/" + f.name for f in (csrc / ".." / ".." / "include").glob("*.h")]
    h = hashlib.sha256()
    for r in sorted(rel):
        h.update((csrc / r).read_bytes())
    return h.hexdigest()[:16]


ALLREDUCE_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64)
COLLECTIVE_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p, ctypes.c_int64)

_lib = None


def load(path: str | os.PathLike | None = None) -> ctypes.CDLL:
    """Load (once) and return the HIP library; raises if it is absent."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = pathlib.Path(path) if path is not None else LIB_PATH
    if not p.exists():
        raise MTSACLibraryError(
            f"{p} not found: build the HIP engine first (python -c 'import __graft_entry__ as g; g.build()')"
        )
    # torch ships its own ROCm runtime (torch/lib/libamdhip64.so, librccl.so, libhsa-runtime64.so)
    # with the same SONAMEs as /opt/rocm.  Import it first so our DT_NEEDED entries bind to the
    # copies already in the process: one HIP/HSA runtime per process, shared with torch.
    if os.environ.get("MTSAC_NO_TORCH_RUNTIME") != "1":
        try:
            import torch  # noqa: F401
        except ImportError:  # pragma: no cover
            pass
    try:
        lib = ctypes.CDLL(str(p), mode=ctypes.RTLD_GLOBAL)
    except OSError as e:  # pragma: no cover - depends on the runtime
        raise MTSACLibraryError(f"failed to load {p}: {e}") from e
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.mtsac_abi_version() != 1:
        raise MTSACLibraryError("libmtsac ABI version mismatch")
    built, tree = lib.mtsac_build_stamp().decode(), source_stamp()
    if tree is not None and built != tree and os.environ.get("MTSAC_ALLOW_STALE_LIB") != "1":
        raise MTSACLibraryError(f"{p} was built from other sources (stamp {built}) than the tree's ({tree}): "
                                "rebuild it (python -c 'import __graft_entry__ as g; g.build()')")
    if path is None:
        _lib = lib
    return lib


def check(rc: int) -> int:
    if rc < 0:
        msg = load().mtsac_last_error()
        raise MTSACError(f"libmtsac error {rc}: {msg.decode() if msg else ''}")
    return rc
