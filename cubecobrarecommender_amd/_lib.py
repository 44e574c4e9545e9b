"""ctypes binding of libccrec_hip.so (include/ccrec.h).  Fails loudly when the library is missing:
there is no CPU fallback anywhere in the product path."""
import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get('CCREC_LIB') or os.path.join(_HERE, 'libccrec_hip.so')

CC_F32, CC_BF16, CC_MX8 = 0, 1, 2
CC_EPI_STORE, CC_EPI_BCE, CC_EPI_MASK, CC_EPI_SPLITK = 0, 1, 2, 3
CC_NUM_TENSORS = 24
CC_KL_DWO_NARROW = 16          # cc_dec_kl_args.flags (dWo's rounding differs: one pass over all rows)


class CCError(RuntimeError):
    pass


class NoiseArgs(C.Structure):
    _fields_ = [
        ('V', C.c_int32), ('B', C.c_int32), ('x_cap', C.c_int32), ('with_reg', C.c_int32),
        ('seed', C.c_uint64), ('slot_base', C.c_uint32), ('batch_stride', C.c_int32),
        ('batch_offset', C.c_int32), ('num_perms', C.c_int32), ('num_cubes', C.c_int32),
        ('noise_mean', C.c_double), ('noise_std', C.c_double),
        ('cube_ptr', C.c_void_p), ('cube_idx', C.c_void_p), ('perm', C.c_void_p),
        ('cdf', C.c_void_p), ('neg_sampler', C.c_void_p), ('guide', C.c_void_p),
        ('guide_log2', C.c_int32), ('state', C.c_void_p),
        ('x_cnt', C.c_void_p), ('x_idx', C.c_void_p), ('y_bits', C.c_void_p),
        ('xt_bits', C.c_void_p), ('reg_idx', C.c_void_p), ('status', C.c_void_p),
        ('xt_rows', C.c_int32), ('reg_slots', C.c_int32), ('reg_lo', C.c_int32),
        ('reg_hi', C.c_int32), ('reg_cap', C.c_int32), ('x_bits', C.c_void_p),
    ]


class GemmArgs(C.Structure):
    _fields_ = [
        ('dtype', C.c_int32), ('ta', C.c_int32), ('tb', C.c_int32), ('epilogue', C.c_int32),
        ('M', C.c_int32), ('N', C.c_int32), ('K', C.c_int32), ('lda', C.c_int32),
        ('ldb', C.c_int32), ('ldc', C.c_int32), ('splits', C.c_int32), ('relu', C.c_int32),
        ('A', C.c_void_p), ('B', C.c_void_p), ('bias', C.c_void_p), ('C', C.c_void_p),
        ('Cf', C.c_void_p), ('H', C.c_void_p), ('y_bits', C.c_void_p), ('scale', C.c_float),
        ('loss_partials', C.c_void_p), ('colsum', C.c_void_p), ('Ct', C.c_void_p), ('ldct', C.c_int32),
        ('loss_out', C.c_void_p), ('loss_scale', C.c_double), ('ticket', C.c_void_p),
        ('a_scale', C.c_void_p), ('b_scale', C.c_void_p),
    ]


class AdamTRegion(C.Structure):
    _fields_ = [('off', C.c_int64), ('rows', C.c_int32), ('cols', C.c_int32), ('dst', C.c_void_p)]


class TowerArgs(C.Structure):
    _fields_ = [
        ('dtype', C.c_int32), ('d', C.c_int32), ('B', C.c_int32), ('R', C.c_int32),
        ('w', C.c_void_p * 9), ('wt', C.c_void_p * 9), ('b', C.c_void_p * 9), ('act', C.c_void_p * 7),
        ('act6t', C.c_void_p),
        ('gD3', C.c_void_p), ('gact', C.c_void_p * 5), ('gpre1', C.c_void_p), ('slab', C.c_void_p),
        ('gw', C.c_void_p * 9), ('gb', C.c_void_p * 9), ('gpre1t', C.c_void_p),
        ('wpf', C.c_void_p * 9), ('wpb', C.c_void_p * 9), ('act6p', C.c_void_p), ('act6tp', C.c_void_p),
        ('hpt', C.c_void_p * 6), ('gpt', C.c_void_p * 6), ('gpre1p', C.c_void_p),
        ('x_bits', C.c_void_p), ('xt_bits', C.c_void_p), ('xt_V', C.c_int32), ('xt_rows', C.c_int32),
        ('d3q', C.c_void_p), ('d3qs', C.c_void_p), ('d3tq', C.c_void_p), ('d3tqs', C.c_void_p),
        ('y_bits', C.c_void_p), ('y_img', C.c_void_p), ('y_V', C.c_int32),
    ]


class DecKlArgs(C.Structure):
    _fields_ = [
        ('d', C.c_int32), ('V', C.c_int32), ('rows', C.c_int32), ('ldt', C.c_int32), ('row0', C.c_int32),
        ('D3p', C.c_void_p), ('D3tp', C.c_void_p), ('Wo', C.c_void_p),
        ('bo', C.c_void_p), ('Mt', C.c_void_p), ('tsum', C.c_void_p), ('mt_bytes', C.c_int64), ('mt_lo', C.c_int32),
        ('reg_idx', C.c_void_p),
        ('scale', C.c_float), ('dZ', C.c_void_p), ('gW', C.c_void_p), ('gb', C.c_void_p),
        ('loss_partials', C.c_void_p), ('loss_out', C.c_void_p), ('loss_scale', C.c_double),
        ('ticket', C.c_void_p), ('ws', C.c_void_p), ('flags', C.c_int32),
    ]


class AdamPack(C.Structure):
    _fields_ = [('n', C.c_int32), ('K', C.c_int32 * 9), ('N', C.c_int32 * 9), ('off', C.c_int64 * 9),
                ('wpf', C.c_void_p * 9), ('wpb', C.c_void_p * 9)]


_P, _I32, _I64, _F32, _F64, _SZ = C.c_void_p, C.c_int32, C.c_int64, C.c_float, C.c_double, C.c_size_t

# name -> (restype, argtypes); every symbol include/ccrec.h declares
SIGNATURES = {
    'cc_abi_version': (C.c_int, []),
    'cc_last_error_string': (C.c_char_p, []),
    'cc_build_id': (C.c_char_p, []),
    'cc_param_layout': (C.c_int, [_I32, _I32, _P, _P, _P, _P]),
    'cc_crc32c': (C.c_uint32, [C.c_uint32, _P, _SZ]),
    'cc_noise_fwd': (C.c_int, [C.POINTER(NoiseArgs), _P]),
    'cc_embed_gather_fwd': (C.c_int, [_I32, _P, _P, _I32, _I32, _I32, _P, _P, _I32, _P, _P]),
    'cc_embed_gather_fwd_warm': (C.c_int, [_I32, _P, _P, _I32, _I32, _I32, _P, _P, _I32, _P, _P, _I64, _P, _I64,
                                           _P]),
    'cc_embed_gather_fwd_xt': (C.c_int, [_I32, _P, _P, _I32, _I32, _I32, _P, _P, _I32, _P, _P, _I64, _P, _I64,
                                         _P, _P, _I32, _P]),
    'cc_embed_scatter_bwd': (C.c_int, [_P, _I32, _I32, _I32, _P, _P, _P, _P]),
    'cc_embed_grad_mfma': (C.c_int, [_P, _I32, _I32, _I32, _I32, _P, _P, _P, _P]),
    'cc_gemm': (C.c_int, [C.POINTER(GemmArgs), _P]),
    'cc_gemm_tile128': (C.c_int, [C.POINTER(GemmArgs), _P]),
    'cc_gemm_pair': (C.c_int, [C.POINTER(GemmArgs), C.POINTER(GemmArgs), _P]),
    'cc_gemm_mx8_wide': (C.c_int, [C.POINTER(GemmArgs), C.POINTER(GemmArgs), _P]),
    'cc_gemm_mx8_bce_q': (C.c_int, [C.POINTER(GemmArgs), _P, C.c_int32, _P, _P, C.c_int32, _P, _P, _P]),
    'cc_gemm_mx8_bce_q2': (C.c_int, [C.POINTER(GemmArgs), _P, C.c_int32, _P, _P, C.c_int32, _P, _P,
                                     C.POINTER(GemmArgs), _P]),
    'cc_gemm_grid': (C.c_int, [_I32, _I32, _P]),
    'cc_splitk_reduce': (C.c_int, [_I32, _P, _I32, _I32, _I32, _P, _P, _P, _P, _P, _P]),
    'cc_splitk_reduce_warm': (C.c_int, [_I32, _P, _I32, _I32, _I32, _P, _P, _P, _P, _P, _P, _I64, _P]),
    'cc_colsum': (C.c_int, [_I32, _P, _I32, _I32, _I32, _P, _P]),
    'cc_transpose': (C.c_int, [_I32, _P, _I32, _I32, _P, _P]),
    'cc_quant_mx8': (C.c_int, [_I32, _P, _I32, _I32, _I32, _I32, _P, _I32, _P, _P, _P]),
    'cc_dec_softmax_kl_q': (C.c_int, [_P, _I32, _I32, _P, _P, _F32, _P, _P, _P, _I32, _P, _P]),
    'cc_quant_mx8_both': (C.c_int, [C.c_int32, _P, C.c_int32, C.c_int32, C.c_int32, _P, C.c_int32, _P, _P, C.c_int32, _P, _P]),
    'cc_dec_bce_fused': (C.c_int, [_I32, _P, _P, _P, _I32, _I32, _I32, _P, _P, _P, _P, _P]),
    'cc_dec_bce_dw': (C.c_int, [_P, _P, _I32, _P, _P, _P, _P, _P, _I32, _I32, _I32, _P, _P, _P, _P, _P, _P, _F64, _P, _P]),
    'cc_dec_bce_dw_ld': (C.c_int, [_P, _P, _I32, _P, _P, _P, _P, _P, _I32, _I32, _I32, _P, _P, _I32, _P, _P, _P,
                                   _P, _F64, _P, _P]),
    'cc_dec_bce_dw_img': (C.c_int, [_P, _P, _I32, _P, _P, _P, _P, _P, _I32, _I32, _I32, _P, _P, _P, _I32, _P, _P,
                                    _P, _P, _F64, _P, _P]),
    'cc_dec_bce_dw_blocks': (_I32, [_I32]),
    'cc_dec_softmax_kl_fused': (C.c_int, [_I32, _P, _I32, _I32, _P, _P, _F32, _P, _P, _P]),
    'cc_reduce_loss': (C.c_int, [_P, _I32, _F64, _P, _P]),
    'cc_gemm_dx_splitk': (C.c_int, [_P, _I32, _P, _I32, _I32, _I32, _I32, _I32, _P, _P]),
    'cc_pack_frag_b_size': (_SZ, [_I32, _I32]),
    'cc_pack_frag_b': (C.c_int, [_P, _I32, _I32, _I32, _P, _P]),
    'cc_gemm_dx_splitk_pk': (C.c_int, [_P, _I32, _P, _I32, _I32, _I32, _I32, _P, _P]),
    'cc_dec_kl_ws_size': (_SZ, [_I32, _I32]),
    'cc_dec_kl_blocks': (_I32, [_I32]),
    'cc_dec_softmax_kl_dw': (C.c_int, [C.POINTER(DecKlArgs), _P]),
    'cc_kl_tsum': (C.c_int, [_P, _I32, _I32, _P, _P]),
    'cc_sigmoid_cat_accuracy': (C.c_int, [_P, _I32, _P, _I32, _I32, _P, _P]),
    'cc_row_argmax': (C.c_int, [_P, _I64, _I32, _I32, _P, _P]),
    'cc_cat_accuracy': (C.c_int, [_P, _I32, _I32, _I32, _P, _P, _I32, _P, _P]),
    'cc_adam_noise': (C.c_int, [_P, _P, _P, _P, _P, _I64, _F32, _F32, _F32, _F32, C.POINTER(NoiseArgs), _I64, _P]),
    'cc_adam_noise_pack2': (C.c_int, [_P, _P, _P, _P, _P, _I64, _I64, _I64, _I64, _F32, _F32, _F32, _F32,
                                      C.POINTER(NoiseArgs), _I64, C.POINTER(AdamPack), _P]),
    'cc_adam_pack2': (C.c_int, [_P, _P, _P, _P, _P, _I64, _I64, _I64, _I64, _F32, _F32, _F32, _F32,
                                C.POINTER(NoiseArgs), _I64, C.POINTER(AdamPack), _P]),
    'cc_adam_noise_pack': (C.c_int, [_P, _P, _P, _P, _P, _I64, _F32, _F32, _F32, _F32, C.POINTER(NoiseArgs), _I64,
                                     C.POINTER(AdamPack), _P]),
    'cc_adam_dense': (C.c_int, [_P, _P, _P, _P, _P, _I64, _P, _F32, _F32, _F32, _F32, _P]),
    'cc_adam_dense_t': (C.c_int, [_P, _P, _P, _P, _P, _I64, _P, _F32, _F32, _F32, _F32, _P, _I32,
                                  _I64, _P]),
    'cc_to_bf16': (C.c_int, [_P, _P, _I64, _P]),
    'cc_state_advance': (C.c_int, [_P, _I64, _P]),
    'cc_infer_encode_ws_size': (_SZ, [_I32, _I32, _I32]),
    'cc_infer_encode_fp32': (C.c_int, [_P, _I32, _I32, _I32, _P, _P, _I32, _P, _P, _P]),
    'cc_infer_decode_fp32': (C.c_int, [_P, _I32, _I32, _I32, _P, _P, _P, _P]),
    'cc_similar_ws_size': (_SZ, [_I32]),
    'cc_similar_cards': (C.c_int, [_P, _I32, _I32, _I32, _I32, _P, _P, _P, _P, _P]),
    'cc_embed_grad_packed': (C.c_int, [_P, _I32, _I32, _I32, _I32, _P, _P, _P, _P]),
    'cc_embed_grad_cs': (C.c_int, [_P, _I32, _I32, _I32, _I32, _I32, _P, _P, _P, _P, _P]),
    'cc_embed_grad_cs_tickets': (_I32, [_I32, _I32, _I32]),
    'cc_embed_grad_cs_adam': (C.c_int, [_P, _I32, _I32, _I32, _I32, _I32, _P, _P, _P, _P, _P, _P, _P, _P,
                                        _F32, _F32, _F32, _F32, _P]),
    'cc_embed_grad_cs_reg': (C.c_int, [_P, _I32, _I32, _I32, _I32, _I32, _P, _P, _P, _P, _P, _I32, _I32, _I32, _P]),
    'cc_embed_grad_cs_adam_reg': (C.c_int, [_P, _I32, _I32, _I32, _I32, _I32, _P, _P, _P, _P, _P, _P, _P, _P,
                                            _F32, _F32, _F32, _F32, _P, _I32, _I32, _P]),
    'cc_embed_identity_ws': (_SZ, [_I32, _I32]),
    'cc_embed_identity_add': (C.c_int, [_I32, _P, _I32, _I32, _I32, _P, _P, _P, _P]),
    'cc_reg_rows': (C.c_int, [C.POINTER(NoiseArgs), _P]),
    'cc_noise_next': (C.c_int, [C.POINTER(NoiseArgs), _I64, _P]),
    'cc_tower_slab_elems': (_I64, [_I32]),
    'cc_tower_fwd': (C.c_int, [C.POINTER(TowerArgs), _P]),
    'cc_tower_bwd': (C.c_int, [C.POINTER(TowerArgs), _P]),
    'cc_tower_bwd_chain': (C.c_int, [C.POINTER(TowerArgs), _P]),
    'cc_tower_bwd_chain_adam': (C.c_int, [C.POINTER(TowerArgs), _P, _P, _P, _P, _P, _I64, _I64, _I64, _I64, _P,
                                          _F32, _F32, _F32, _F32, _P]),
    'cc_tower_bwd_chain_noise': (C.c_int, [C.POINTER(TowerArgs), C.POINTER(NoiseArgs), _I64, _P, _P, _P, _P, _P,
                                           _I64, _I64, _I64, _I64, _P, _F32, _F32, _F32, _F32, _P]),
    'cc_tower_bwd_dw': (C.c_int, [C.POINTER(TowerArgs), _P]),
    'cc_tower_reduce': (C.c_int, [C.POINTER(TowerArgs), _P]),
    'cc_tower_transpose': (C.c_int, [C.POINTER(TowerArgs), _P]),
    'cc_tower_bwd_dw_direct': (C.c_int, [C.POINTER(TowerArgs), _P]),
    'cc_tower_transpose_advance': (C.c_int, [C.POINTER(TowerArgs), _P, _I64, _P]),
    'cc_topn_workspace_size': (_SZ, [_I32]),
    'cc_topn': (C.c_int, [_P, _I32, _P, _I32, _I32, _P, _P, _P, _P, _P, _P, _P]),
    'cc_recommend_ws_size': (_SZ, [_I32, _I32]),
    'cc_recommend_fp32': (C.c_int, [_P, _I32, _I32, _P, _I32, _P, _P, _P, _P]),
    'cc_recommend_graph_create': (C.c_int, [_P, _I32, _I32, _P, _P, _I32, _P, _P, _P, C.POINTER(C.c_void_p)]),
    'cc_recommend_graph_run': (C.c_int, [_P, _P, _I32]),
    'cc_recommend_graph_destroy': (C.c_int, [_P]),
    'cc_adjacency_ws_size': (_SZ, [_I32, _I32, _I32, _I32]),
    'cc_adjacency': (C.c_int, [_P, _P, _I32, _I32, _I32, _P, _P, _P, _P, _P, _P]),
}

_lib = None


def lib():
    """Load (once) and return the library with typed entry points."""
    global _lib
    if _lib is None:
        # Load torch (and with it PyTorch's HIP runtime) first so libccrec_hip binds to the same
        # libamdhip64 instance as the tensors it is handed; a second HIP runtime in the process
        # sees no device.
        import torch  # noqa: F401
        if not os.path.exists(LIB_PATH):
            raise CCError(f'libccrec_hip.so not found at {LIB_PATH}; build it with '
                          f'`python -m cubecobrarecommender_amd.build` (no CPU fallback exists)')
        L = C.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        if L.cc_abi_version() != 2:
            raise CCError('libccrec_hip ABI version mismatch')
        _lib = L
    return _lib


def check_build_id():
    """Raise unless the loaded library was compiled from the sources in this tree (buildid.py):
    tests/conftest.py and __graft_entry__.smoke() call it so no result rests on a stale binary."""
    from .buildid import tree_build_id
    got = lib().cc_build_id().decode()
    want = tree_build_id()
    if got != want:
        raise CCError(f'{LIB_PATH} was built from other sources (build id {got}, tree {want}): '
                      f'rebuild with `python -m cubecobrarecommender_amd.build`')
    return got


def check(rc, what=''):
    if rc != 0:
        msg = lib().cc_last_error_string()
        raise CCError(f'{what} failed ({rc}): {msg.decode() if msg else ""}')


def call(name, *args):
    check(getattr(lib(), name)(*args), name)


def ptr(t):
    """Device pointer of a torch tensor (None -> NULL)."""
    return None if t is None else C.c_void_p(t.data_ptr())


def stream_ptr(stream=None):
    import torch
    s = stream if stream is not None else torch.cuda.current_stream()
    return C.c_void_p(s.cuda_stream)
