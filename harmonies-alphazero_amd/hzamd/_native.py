"""ctypes binding of libhz.so (include/hz_abi.h).

The product path has no CPU fallback: if the HIP library is missing or was
built for another architecture, `lib()` raises.  torch is imported first so
that libhz.so binds to the HIP runtime torch already loaded (both carry the
soname libamdhip64.so.7), which keeps torch device pointers valid here.
"""
import ctypes
import os

import torch  # noqa: F401  (must precede the CDLL load, see module docstring)

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.environ.get("HZ_LIB") or os.path.join(PKG_DIR, "libhz.so")  # HZ_LIB: diagnostic builds

_lib = None

_c = ctypes
_vp = ctypes.c_void_p
_SIGS = {
    "hz_env_create": ([_c.c_int32, _c.c_uint64, _vp], _vp),
    "hz_env_destroy": ([_vp], None),
    "hz_env_size": ([_vp], _c.c_int32),
    "hz_env_set_stream": ([_vp, _vp], _c.c_int),
    "hz_env_state_ptr": ([_vp], _vp),
    "hz_env_mt_ptr": ([_vp], _vp),
    "hz_env_mt_pos_ptr": ([_vp], _vp),
    "hz_env_ply_ptr": ([_vp], _vp),
    "hz_env_seed_ptr": ([_vp], _vp),
    "hz_reset": ([_vp, _vp, _vp], _c.c_int),
    "hz_legal_mask": ([_vp, _vp, _vp], _c.c_int),
    "hz_legal_actions": ([_vp, _vp, _vp], _c.c_int),
    "hz_step": ([_vp, _vp, _vp], _c.c_int),
    "hz_score": ([_vp, _vp, _vp], _c.c_int),
    "hz_replenish": ([_vp, _vp], _c.c_int),
    "hz_end_turn": ([_vp, _vp], _c.c_int),
    "hz_encode": ([_vp, _vp, _c.c_int32, _vp, _vp], _c.c_int),
    "hz_rule_actions": ([_vp, _vp, _vp, _vp], _c.c_int),
    "hz_rule_ply": ([_vp, _vp, _vp, _vp, _vp], _c.c_int),
    "hz_encode_states": ([_vp, _c.c_int64, _c.c_int64, _vp, _c.c_int32, _vp, _vp, _vp], _c.c_int),
    "hz_rollout": ([_vp, _c.c_int32, _c.c_int32, _vp, _vp, _vp, _vp, _vp], _c.c_int),
    "hz_play": ([_vp, _c.c_int32, _c.c_int32, _vp, _vp, _vp, _vp, _vp], _c.c_int),
    "hz_env_set_seed_ahead": ([_vp, _c.c_int32], _c.c_int),
    "hz_env_set_auto_ahead": ([_vp, _c.c_int32], _c.c_int),
    "hz_env_set_pipeline": ([_vp, _c.c_int32], _c.c_int),
    "hz_env_set_error_word": ([_vp, _vp], _c.c_int),
    "hz_env_set_spin_limit": ([_vp, _c.c_int32], _c.c_int),
    "hz_greedy_actions": ([_vp, _vp, _vp], _c.c_int),
    "hz_export_state": ([_vp, _vp, _vp, _vp], _c.c_int),
    "hz_import_state": ([_vp, _vp, _vp, _vp], _c.c_int),
    "hz_mcts_create": ([_c.c_int32, _c.c_int32, _c.c_int32, _c.c_int32, _vp], _vp),
    "hz_mcts_destroy": ([_vp], None),
    "hz_mcts_set_stream": ([_vp, _vp], _c.c_int),
    "hz_mcts_begin": ([_vp, _vp, _vp], _c.c_int),
    "hz_mcts_select": ([_vp, _vp, _c.c_float], _c.c_int),
    "hz_mcts_encode_leaves": ([_vp, _vp, _vp], _c.c_int),
    "hz_mcts_expand_backup": ([_vp, _vp, _vp, _vp, _vp, _c.c_double, _c.c_int32], _c.c_int),
    "hz_mcts_gather_leaves": ([_vp, _vp, _vp, _vp, _vp], _c.c_int),
    "hz_mcts_set_eval_counter": ([_vp, _vp], _c.c_int),
    "hz_mcts_set_dedup_walk": ([_vp, _c.c_int32], _c.c_int),
    "hz_mcts_set_gather_encode": ([_vp, _c.c_int32], _c.c_int),
    "hz_mcts_select_gather": ([_vp, _vp, _c.c_float, _vp, _vp, _vp, _vp], _c.c_int),
    "hz_mcts_expand_backup_gathered": ([_vp, _vp, _vp, _vp, _vp, _c.c_double, _c.c_int32], _c.c_int),
    "hz_mcts_expand_backup_select": ([_vp, _vp, _vp, _vp, _vp, _c.c_double, _c.c_int32, _vp, _c.c_float], _c.c_int),
    "hz_mcts_expand_backup_select_gather": ([_vp, _vp, _vp, _vp, _vp, _c.c_double, _c.c_int32, _vp, _c.c_float,
                                             _vp, _vp, _vp, _vp, _vp, _c.c_int32], _c.c_int),
    "hz_mcts_result": ([_vp, _vp], _c.c_int),
    "hz_root_noise": ([_vp, _c.c_int32, _c.c_uint64, _c.c_uint64, _c.c_uint64, _c.c_double, _vp, _vp, _vp],
                      _c.c_int),
    "hz_mcts_stats": ([_vp, _vp], _c.c_int),
    "hz_mcts_leaf_ptrs": ([_vp, _vp, _vp], _c.c_int),
    "hz_mcts_path_edges": ([_vp, _vp], _c.c_int),
    "hz_bias_act": ([_vp, _vp, _vp, _c.c_int64, _c.c_int32, _vp], _c.c_int),
    "hz_conv3x3_bias_act": ([_vp, _vp, _vp, _vp, _vp, _c.c_int32, _vp, _vp], _c.c_int),
    "hz_heads": ([_vp, _vp, _vp, _vp, _vp, _vp, _c.c_int32, _vp, _vp], _c.c_int),
    "hz_heads_fc": ([_vp] * 13 + [_c.c_int32, _vp, _vp], _c.c_int),
    "hz_conv3x3_x6_bias_act": ([_vp, _vp, _vp, _vp, _vp, _c.c_int32, _vp, _vp], _c.c_int),
    "hz_stem3x3_x6_bias_act": ([_vp, _vp, _vp, _vp, _c.c_int32, _vp, _vp], _c.c_int),
    "hz_resblock_x6_bias_act": ([_vp, _vp, _vp, _vp, _vp, _vp, _vp, _c.c_int32, _vp, _vp], _c.c_int),
    "hz_resblock_x6_fused": ([_c.c_int32], _c.c_int32),
    "hz_resblock_x6_set_fused": ([_c.c_int32], _c.c_int),
    "hz_resblock_x6_set_table": ([_c.c_int32], _c.c_int),
    "hz_tower_x6_set_stagger": ([_c.c_int32], _c.c_int),
    "hz_tower_x6_blocks": ([_vp, _vp, _vp, _vp, _vp, _c.c_int32, _vp, _vp, _c.c_int32, _vp, _vp], _c.c_int),
    "hz_tower_x6_resident": ([_vp, _vp, _vp, _vp, _c.c_int32, _c.c_int32, _vp, _vp], _c.c_int),
    "hz_tower_x6_split": ([_vp, _vp, _vp, _vp, _vp, _vp, _c.c_int32, _c.c_int32, _vp, _vp], _c.c_int),
    "hz_tower_x6_split_max_batch": ([], _c.c_int32),
    "hz_tower_x6_split_set_limit": ([_c.c_int32], _c.c_int),
    "hz_stem3x3_bias_act": ([_vp, _vp, _vp, _vp, _c.c_int32, _vp, _vp], _c.c_int),
    "hz_version": ([], _c.c_char_p),
}


class NativeError(RuntimeError):
    pass


def exported_symbols():
    return sorted(_SIGS)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise NativeError(
                f"libhz.so not found at {LIB_PATH}: build it with __graft_entry__.build() "
                "(hipcc --offload-arch=gfx950); there is no CPU fallback")
        L = ctypes.CDLL(LIB_PATH)
        for name, (args, res) in _SIGS.items():
            try:
                fn = getattr(L, name)
            except AttributeError:
                # an older build named by HZ_LIB (A/B tools) may predate a
                # symbol; the in-tree library must export every one
                if os.environ.get("HZ_LIB"):
                    continue
                raise
            fn.argtypes = args
            fn.restype = res
        _lib = L
    return _lib


def check(rc, what):
    if rc != 0:
        raise NativeError(f"{what} failed with code {rc}")


def ptr(t):
    """Device pointer of a torch tensor (None -> NULL)."""
    if t is None:
        return None
    return ctypes.c_void_p(t.data_ptr())


def stream_ptr(device=None):
    s = torch.cuda.current_stream(device)
    return ctypes.c_void_p(s.cuda_stream)
