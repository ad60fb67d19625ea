"""ctypes binding of ``libwc_kernels.so`` (the C ABI declared in ``include/wc_kernels.h``).

There is deliberately no CPU fallback: every product entry point goes through these kernels and a
missing or failing library raises.  ``torch`` is imported before the library is opened so the HIP
runtime torch ships (soname ``libamdhip64.so.7``) is the one the kernels bind to.
"""
import contextlib
import ctypes
import os
import threading

import torch  # noqa: F401  (loads the HIP runtime first)

from . import _build

MAX_TAPS = 16
NOISE_NONE, NOISE_TENSOR, NOISE_PHILOX = 0, 1, 2

EXPORTS = [
    'wc_conv_igemm', 'wc_conv3x3_x6', 'wc_conv3x3_f16x3', 'wc_conv3x3_wino_f16x3', 'wc_conv3x3_wino_tile_n', 'wc_wino_vsplit_bytes', 'wc_wino_vsplit_f16x3', 'wc_conv3x3_wino_f16x3_vp', 'wc_conv3x3_wino_f16x3_vp8', 'wc_conv3x3_wino_gnb_splits', 'wc_conv3x3_wino_f16x3_gnb', 'wc_pack_wino', 'wc_pack_wino_raw', 'wc_pack_wino_batch', 'wc_conv3x3_x6_tile_n', 'wc_conv_igemm_x6',
    'wc_conv_igemm_f16x3', 'wc_conv4x4s2_f16x3', 'wc_convtr4x4s2_f16x3', 'wc_conv_igemm_f16x3_qkv', 'wc_split_f16x3_tiled', 'wc_attention_fwd_f16x3_presplit_a3', 'wc_proj_f16x3', 'wc_proj_f16x3_qkv', 'wc_proj_set_tile', 'wc_attention_fwd_f16x3_presplit',
    'wc_gn_num_splits',
    'wc_gn_stats', 'wc_gn_finalize', 'wc_gn_finalize_bound', 'wc_gn_partials', 'wc_gn_finalize_part', 'wc_attention_fwd', 'wc_attention_fwd_x6', 'wc_attention_fwd_f16x3',
    'wc_temb', 'wc_conv_in', 'wc_conv_in_gn', 'wc_head_conv', 'wc_ddpm_step', 'wc_add_noise', 'wc_philox_normal', 'wc_sgg_update',
    'wc_avgpool2x2', 'wc_upsample2x_bilinear', 'wc_layernorm_channels', 'wc_noise_embed',
    'wc_mse_workspace_doubles', 'wc_mse_loss', 'wc_dwconv', 'wc_version', 'wc_source_hash',
    'wc_conv_wgrad', 'wc_conv_wgrad_x6', 'wc_conv_wgrad_f16x3', 'wc_conv_wgrad_splits', 'wc_wgrad_reduce', 'wc_gn_bwd_splits', 'wc_gn_bwd_reduce',
    'wc_gn_bwd_finalize', 'wc_bsum', 'wc_bsum_batch', 'wc_gn_bwd_apply', 'wc_attention_fwd_lse', 'wc_attention_bwd', 'wc_gemm_small',
    'wc_silu', 'wc_colsum', 'wc_time_embedding', 'wc_nchw_to_nhwc', 'wc_last_kernel_name', 'wc_stamp', 'wc_wall_clock_khz',
    'wc_attention_fwd_f16x3_lse', 'wc_attention_fwd_x6_lse',
    'wc_conv_wgrad3', 'wc_conv_wgrad3_f16x3', 'wc_conv_wgrad3_splits', 'wc_absmax_images', 'wc_attention_bwd6', 'wc_attention_bwd_f16x3', 'wc_attention_bwd_dkdv192', 'wc_attention_bwd_prep', 'wc_pack_split',
    'wc_small_wgrad_workspace', 'wc_head_dgrad', 'wc_head_wgrad', 'wc_stem_wgrad'
]
ACT_NONE, ACT_GELU, ACT_SILU, ACT_PRELU, ACT_TANH01 = 0, 1, 2, 3, 4


class ConvSeg(ctypes.Structure):
    _fields_ = [
        ('src', ctypes.c_void_p), ('C', ctypes.c_int), ('ldc', ctypes.c_int), ('H', ctypes.c_int),
        ('W', ctypes.c_int), ('sy', ctypes.c_int), ('sx', ctypes.c_int), ('ntaps', ctypes.c_int),
        ('dy', ctypes.c_int * MAX_TAPS), ('dx', ctypes.c_int * MAX_TAPS), ('scale', ctypes.c_void_p),
        ('shift', ctypes.c_void_p), ('silu', ctypes.c_int), ('kbase', ctypes.c_int)
    ]


class GnbEpi(ctypes.Structure):
    """wc_gnb_epi (include/wc_kernels.h): the GroupNorm-backward sums a data-gradient conv's epilogue forms."""
    _fields_ = [('x', ctypes.c_void_p), ('ldx', ctypes.c_int), ('silu', ctypes.c_int), ('sc0', ctypes.c_void_p),
                ('sh0', ctypes.c_void_p), ('gamma', ctypes.c_void_p), ('beta', ctypes.c_void_p),
                ('part', ctypes.c_void_p), ('part3', ctypes.c_void_p), ('splits', ctypes.c_int), ('pad', ctypes.c_int)]


class ConvArgs(ctypes.Structure):
    _fields_ = [
        ('seg', ConvSeg * 2), ('nseg', ctypes.c_int), ('B', ctypes.c_int), ('Hm', ctypes.c_int),
        ('Wm', ctypes.c_int), ('N', ctypes.c_int), ('w', ctypes.c_void_p), ('ldw', ctypes.c_int),
        ('bias', ctypes.c_void_p), ('temb', ctypes.c_void_p), ('temb_ld', ctypes.c_int),
        ('res', ctypes.c_void_p), ('ldres', ctypes.c_int), ('out', ctypes.c_void_p),
        ('ldo', ctypes.c_int), ('Ho', ctypes.c_int), ('Wo', ctypes.c_int), ('osy', ctypes.c_int),
        ('osx', ctypes.c_int), ('ooy', ctypes.c_int), ('oox', ctypes.c_int),
        ('out_nchw', ctypes.c_int), ('act', ctypes.c_int), ('absmax_out', ctypes.c_void_p),
        ('act_param', ctypes.c_void_p), ('gn_part', ctypes.c_void_p), ('gn_ncb', ctypes.c_int),
        ('gn_sw', ctypes.c_int), ('gn_c0', ctypes.c_int), ('gn_p64', ctypes.c_int), ('gn_np64', ctypes.c_int)
    ]


class WgradArgs(ctypes.Structure):
    _fields_ = [
        ('g', ctypes.c_void_p), ('M', ctypes.c_int), ('ldg', ctypes.c_int), ('seg', ConvSeg * 2),
        ('nseg', ctypes.c_int), ('B', ctypes.c_int), ('Hm', ctypes.c_int), ('Wm', ctypes.c_int)
    ]


_P = ctypes.c_void_p
_I = ctypes.c_int
_L = ctypes.c_int64
_F = ctypes.c_float
_D = ctypes.c_double
_U = ctypes.c_uint64

_SIGS = {
    'wc_conv_igemm': [ctypes.POINTER(ConvArgs), _P],
    'wc_conv3x3_x6': [ctypes.POINTER(ConvArgs), _P, _L, _P],
    'wc_conv3x3_x6_tile_n': [_I],
    'wc_proj_set_tile': [_I],
    'wc_conv3x3_f16x3': [ctypes.POINTER(ConvArgs), _P, _L, _I, _P, _P, _P],
    'wc_conv3x3_wino_f16x3': [ctypes.POINTER(ConvArgs), _P, _L, _I, _P, _P, _P],
    'wc_wino_vsplit_bytes': [_I, _I, _I, _I, _P],
    'wc_wino_vsplit_f16x3': [ctypes.POINTER(ConvArgs), _I, _P, _P, _L, _P],
    'wc_conv3x3_wino_f16x3_vp': [ctypes.POINTER(ConvArgs), _P, _L, _I, _P, _P, _P, _L, _P],
    'wc_conv3x3_wino_f16x3_vp8': [ctypes.POINTER(ConvArgs), _P, _L, _I, _P, _P, _P, _L, _P],
    'wc_conv3x3_wino_tile_n': [_I],
    'wc_conv3x3_wino_gnb_splits': [_I, _I, _I],
    'wc_conv3x3_wino_f16x3_gnb': [ctypes.POINTER(ConvArgs), _P, _L, _I, _P, _P, ctypes.POINTER(GnbEpi), _P],
    'wc_pack_wino': [_P, _I, _I, _I, _P, _L, _P, _P],
    'wc_pack_wino_raw': [_P, _P, _I, _I, _I, _I, _P, _L, _P, _P],
    'wc_pack_wino_batch': [_P, _I, _I, _I, _P],
    'wc_conv_igemm_x6': [ctypes.POINTER(ConvArgs), _P, _L, _P],
    'wc_conv_igemm_f16x3': [ctypes.POINTER(ConvArgs), _P, _L, _I, _P, _P, _P],
    'wc_conv4x4s2_f16x3': [ctypes.POINTER(ConvArgs), _P, _L, _P, _P, _P],
    'wc_convtr4x4s2_f16x3': [ctypes.POINTER(ConvArgs), _P, _L, _P, _P, _P],
    'wc_conv_igemm_f16x3_qkv': [ctypes.POINTER(ConvArgs), _P, _L, _I, _P, _P, _I, _I, _P, _P],
    'wc_split_f16x3_tiled': [_P, _I, _I, _I, _I, _P, _P, _I, _I, _P, _L, _P],
    'wc_attention_fwd_f16x3_presplit_a3': [_P, _P, _L, _I, _I, _I, _I, _F, _I, _I, _I, _P],
    'wc_proj_f16x3': [ctypes.POINTER(ConvArgs), _P, _L, _P, _L, _I, _P, _P],
    'wc_proj_f16x3_qkv': [ctypes.POINTER(ConvArgs), _P, _L, _P, _L, _I, _P, _P, _I, _I, _P, _P],
    'wc_attention_fwd_f16x3_presplit': [_P, _P, _I, _I, _I, _I, _I, _F, _I, _I, _I, _P],
    'wc_gn_num_splits': [_I, _I, _I],
    'wc_stamp': [_P, _I, _P],
    'wc_wall_clock_khz': [_P],
    'wc_gn_stats': [_P, _I, _I, _I, _I, _I, _P, _P],
    'wc_gn_finalize': [_P, _I, _I, _I, _I, _P, _P, _F, _P, _P, _P],
    'wc_gn_finalize_bound': [_P, _I, _I, _I, _I, _P, _P, _F, _P, _P, _P, _P],
    'wc_gn_partials': [_P, _I, _I, _I, _I, _P, _I, _I, _I, _P],
    'wc_gn_finalize_part': [_P, _I, _I, _I, _I, _I, _I, _I, _P, _P, _F, _P, _P, _P, _P],
    'wc_attention_fwd': [_P, _I, _P, _I, _I, _I, _I, _I, _F, _P],
    'wc_attention_fwd_x6': [_P, _I, _P, _I, _I, _I, _I, _I, _F, _P],
    'wc_attention_fwd_f16x3': [_P, _I, _P, _I, _I, _I, _I, _I, _F, _I, _I, _I, _P],
    'wc_attention_fwd_f16x3_lse': [_P, _I, _P, _I, _P, _I, _I, _I, _I, _F, _I, _I, _I, _P],
    'wc_attention_fwd_x6_lse': [_P, _I, _P, _I, _P, _I, _I, _I, _I, _F, _P],
    'wc_temb': [_P, _I, _I, _P, _P, _P, _P, _P, _P, _I, _P, _P],
    'wc_conv_in': [_P, _I, _I, _I, _I, _P, _P, _I, _P, _I, _P],
    'wc_conv_in_gn': [_P, _I, _I, _I, _I, _P, _P, _I, _P, _I, _P, _I, _I, _I, _P],
    'wc_head_conv': [_P, _I, _P, _P, _I, _I, _I, _I, _P, _P, _I, _P, _P],
    'wc_ddpm_step': [_P, _P, _P, _P, _P, _L, _L, _F, _F, _F, _F, _I, _U, _L, _L, _P],
    'wc_add_noise': [_P, _P, _P, _P, _P, _L, _L, _P],
    'wc_philox_normal': [_P, _L, _L, _U, _L, _L, _P],
    'wc_sgg_update': [_P, _P, _P, _P, _P, _I, _I, _F, _D, _D, _D, _I, _P],
    'wc_avgpool2x2': [_P, _I, _P, _I, _I, _I, _I, _I, _P],
    'wc_upsample2x_bilinear': [_P, _I, _P, _I, _I, _I, _I, _I, _P],
    'wc_layernorm_channels': [_P, _I, _P, _P, _F, _P, _I, _L, _I, _P],
    'wc_noise_embed': [_P, _P, _I, _P, _I, _I, _I, _P],
    'wc_mse_workspace_doubles': [],
    'wc_mse_loss': [_P, _P, _L, _P, _F, _P, _P, _P],
    'wc_dwconv': [_P, _I, _P, _I, _P, _P, _I, _I, _I, _I, _I, _P],
    'wc_small_wgrad_workspace': [_I, _I, _I, _I],
    'wc_head_dgrad': [_P, _I, _I, _I, _I, _P, _I, _P, _I, _P],
    'wc_head_wgrad': [_P, _I, _P, _P, _P, _I, _I, _I, _I, _I, _P, _L, _P, _I, _P],
    'wc_stem_wgrad': [_P, _I, _P, _I, _I, _I, _I, _I, _P, _L, _P, _I, _P],
    'wc_conv_wgrad': [ctypes.POINTER(WgradArgs), _P, _I, _P],
    'wc_conv_wgrad_x6': [ctypes.POINTER(WgradArgs), _P, _I, _P],
    'wc_conv_wgrad_f16x3': [ctypes.POINTER(WgradArgs), _P, _I, _P, _I, _P, _P, _P],
    'wc_conv_wgrad_splits': [_I, _I, _L, _I],
    'wc_conv_wgrad3': [ctypes.POINTER(WgradArgs), _P, _I, _P],
    'wc_conv_wgrad3_f16x3': [ctypes.POINTER(WgradArgs), _P, _I, _I, _P, _P],
    'wc_conv_wgrad3_splits': [_I, _I, _I, _I, _I, _I],
    'wc_absmax_images': [_P, _I, _I, _I, _I, _P, _P],
    'wc_attention_bwd6': [_P, _I, _P, _I, _P, _I, _P, _P, _P, _I, _I, _I, _I, _I, _F, _P],
    'wc_attention_bwd_f16x3': [_P, _I, _P, _I, _P, _I, _P, _P, _P, _I, _I, _I, _I, _I, _F, _I, _I, _I, _P, _P, _P],
    'wc_attention_bwd_dkdv192': [_P, _I, _P, _I, _P, _P, _P, _I, _I, _I, _I, _I, _F, _P],
    'wc_attention_bwd_prep': [_P, _I, _P, _I, _I, _I, _I, _I, _P, _P],
    'wc_pack_split': [_P, _I, _I, _I, _I, _I, _I, _I, _I, _I, _P, _L, _P, _P],
    'wc_wgrad_reduce': [_P, _I, _I, _I, _I, _I, _I, _P, _L, _L, _L, _P, _L, _I, _P],
    'wc_gn_bwd_splits': [_I, _I],
    'wc_gn_bwd_reduce': [_P, _I, _P, _I, _P, _P, _P, _P, _I, _I, _I, _I, _I, _P, _P, _P],
    'wc_gn_bwd_finalize': [_P, _I, _I, _I, _I, _I, _P, _P, _P, _P, _P, _P, _P],
    'wc_bsum': [_P, _I, _I, _I, _P, _I, _P],
    'wc_bsum_batch': [_P, _I, _I, _I, _P],
    'wc_gn_bwd_apply': [_P, _I, _P, _I, _P, _P, _P, _P, _I, _P, _I, _I, _I, _P, _I, _I, _P, _P],
    'wc_attention_fwd_lse': [_P, _I, _P, _I, _P, _I, _I, _I, _I, _F, _P],
    'wc_attention_bwd': [_P, _I, _P, _I, _P, _I, _P, _P, _P, _I, _I, _I, _I, _I, _F, _P],
    'wc_gemm_small': [_I, _I, _I, _P, _L, _L, _P, _L, _L, _P, _L, _F, _F, _P],
    'wc_silu': [_P, _P, _P, _L, _I, _P],
    'wc_colsum': [_P, _I, _I, _L, _P, _I, _P],
    'wc_time_embedding': [_P, _I, _I, _P, _P],
    'wc_nchw_to_nhwc': [_P, _I, _I, _I, _I, _P, _I, _P],
}

_libs = {}
_active = threading.local()


def lib_path(variant: str = '') -> str:
    """The in-tree library (variant 'single16' / 'bf16': the single-piece builds); WC_KERNEL_LIB
    (WC_KERNEL_LIB_SINGLE16, WC_KERNEL_LIB_BF16) points at another build of it (developer A/B runs only,
    with WC_ALLOW_STALE_LIB=1)."""
    if variant == 'single16':
        return os.environ.get('WC_KERNEL_LIB_SINGLE16', _build.SINGLE16_LIB_PATH)
    if variant == 'bf16':
        return os.environ.get('WC_KERNEL_LIB_BF16', _build.BF16_LIB_PATH)
    return os.environ.get('WC_KERNEL_LIB', _build.LIB_PATH)


@contextlib.contextmanager
def variant(name: str):
    """Route every kernel call of this thread to a library variant inside the block ('' = default,
    'single16' = the single-piece f16 build, 'bf16' = the single-piece bf16 build).  Both libraries stay loaded side by side (RTLD_LOCAL)."""
    prev = getattr(_active, 'v', '')
    _active.v = name
    try:
        yield
    finally:
        _active.v = prev


def active_variant() -> str:
    """The library variant the calling thread's kernel calls go to ('' = the default build)."""
    return getattr(_active, 'v', '')


def load(build_if_missing: bool = True):
    """Open the kernel library of the active variant (building it first if it is absent and hipcc
    exists)."""
    v = getattr(_active, 'v', '')
    lib = _libs.get(v)
    if lib is not None:
        return lib
    path = lib_path(v)
    if not os.path.exists(path):
        if not build_if_missing or not os.path.exists(_build.HIPCC):
            raise RuntimeError(f'weatherconverter_amd: HIP kernel library missing at {path}; run '
                               f'python -c "import __graft_entry__ as g; g.build()"')
        _build.build()
    lib = ctypes.CDLL(path)
    verify_source_hash(lib, v)
    stale_ok = os.environ.get('WC_ALLOW_STALE_LIB', '0') == '1'
    for name, argtypes in _SIGS.items():
        if stale_ok and not hasattr(lib, name):  # an older A/B build may lack newer entry points
            continue
        fn = getattr(lib, name)
        fn.argtypes = argtypes
        fn.restype = ctypes.c_int
    if hasattr(lib, 'wc_small_wgrad_workspace'):
        lib.wc_small_wgrad_workspace.restype = ctypes.c_int64
    lib.wc_version.argtypes = []
    lib.wc_version.restype = ctypes.c_char_p
    lib.wc_last_kernel_name.argtypes = []
    lib.wc_last_kernel_name.restype = ctypes.c_char_p
    for name, value in _selectors.items():  # kernel-form selectors set before this variant was opened
        if hasattr(lib, name) or not stale_ok:
            getattr(lib, name)(value)
    _libs[v] = lib
    return lib


_VARIANT_FLAG = {'': '', 'single16': '1', 'bf16': '2'}


def verify_source_hash(lib, variant: str = ''):
    """Refuse a library built from other sources than this tree's: its compiled-in digest
    (wc_source_hash) must equal _build.source_hash() of the tree's csrc/, header and flags.
    WC_ALLOW_STALE_LIB=1 lets a developer run a deliberately different build (an A/B variant)."""
    stale_ok = os.environ.get('WC_ALLOW_STALE_LIB', '0') == '1'
    if not hasattr(lib, 'wc_source_hash'):
        if stale_ok:  # an older A/B build from before the digest existed
            return None
        raise RuntimeError('weatherconverter_amd: kernel library has no wc_source_hash (built from other sources)')
    lib.wc_source_hash.argtypes = []
    lib.wc_source_hash.restype = ctypes.c_char_p
    got = lib.wc_source_hash().decode()
    want = _build.source_hash(_VARIANT_FLAG.get(variant, ''))
    if got != want and not stale_ok:
        raise RuntimeError(f'weatherconverter_amd: kernel library {variant or "default"} was built from other sources '
                           f'(library digest {got}, tree digest {want}); rebuild with '
                           f'python -c "import __graft_entry__ as g; g.build()" (or set WC_ALLOW_STALE_LIB=1 for a '
                           f'deliberate A/B build)')
    return got


# Process-wide kernel-form selectors (wc_proj_set_tile): each library variant
# keeps its own static state, so a setting is applied to every loaded variant and replayed into any
# variant opened later (the single16 training line included).
_selectors = {}


def set_selector(name: str, value: int, valid=lambda prev: True) -> int:
    """Apply selector `name` (an int -> previous-int entry point) to every library variant; returns the
    previous value of the active variant's (a result `valid` rejects raises, and nothing is applied)."""
    prev = getattr(load(), name)(int(value))
    if not valid(prev):
        raise RuntimeError(f'weatherconverter_amd kernel {name} failed: bad argument {value}')
    for lib in list(_libs.values()):
        if lib is not load():
            getattr(lib, name)(int(value))
    _selectors[name] = int(value)
    return prev


def check(status: int, op: str):
    if status != 0:
        kind = {-1: 'unsupported shape', -2: 'bad argument'}.get(status, f'hipError {status}')
        raise RuntimeError(f'weatherconverter_amd kernel {op} failed: {kind}')


def call(name: str, *args):
    check(getattr(load(), name)(*args), name)


def last_kernel_name() -> str:
    """The exact instantiation (rocprofv3's name) of the kernel the last named launcher started on
    this thread, or '' (wc_last_kernel_name)."""
    return load().wc_last_kernel_name().decode()
