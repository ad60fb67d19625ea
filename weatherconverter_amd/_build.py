"""Build ``libwc_kernels.so`` in-tree with hipcc for gfx950.

The library is a plain C-ABI shared object (no torch symbols), loaded through ctypes by
``weatherconverter_amd._native``.  It links the HIP runtime by soname (``libamdhip64.so.7``); at run
time the copy torch already loaded is reused, so there is exactly one HIP runtime per process.
"""
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, 'csrc')
LIBDIR = os.path.join(HERE, 'lib')
LIBNAME = 'libwc_kernels.so'
LIB_PATH = os.path.join(LIBDIR, LIBNAME)
ROOT = os.path.dirname(HERE)

HIPCC = os.environ.get('HIPCC', '/opt/rocm/bin/hipcc')
ARCH = os.environ.get('WC_OFFLOAD_ARCH', 'gfx950')

SOURCES = ['wc_conv.hip', 'wc_conv6.hip', 'wc_igemm6.hip', 'wc_gn.hip', 'wc_attention.hip', 'wc_attention6.hip', 'wc_misc.hip', 'wc_old.hip', 'wc_train.hip', 'wc_srgan.hip', 'wc_backward.hip', 'wc_attention_bwd.hip', 'wc_wgrad3.hip', 'wc_attention_bwd6.hip', 'wc_pack.hip', 'wc_wino.hip']
HEADERS = ['wc_common.hpp', 'wc_x6.hpp']
# The single-piece build (the 16-bit training line): the sources holding f16x3 correction products
# recompiled with -DWC_SINGLE16=1 (wc_x6.hpp: mfma_f16c), every other object shared.
SINGLE16_SOURCES = ['wc_conv6.hip', 'wc_igemm6.hip', 'wc_attention6.hip', 'wc_wgrad3.hip', 'wc_backward.hip',
                    'wc_attention_bwd6.hip', 'wc_wino.hip', 'wc_pack.hip']
SINGLE16_LIB_PATH = os.path.join(LIBDIR, 'libwc_kernels_single16.so')
# The bf16 single-piece build (the bf16 training line, BASELINE config 3): the same sources with
# -DWC_SINGLE16=2 (bf16 pieces on the bf16 MFMA; packs and pre-split writers emit bf16 bits).
BF16_LIB_PATH = os.path.join(LIBDIR, 'libwc_kernels_bf16.so')

CFLAGS = [
    '-O3', '-std=c++17', '-fPIC', f'--offload-arch={ARCH}', '-munsafe-fp-atomics',
    '-I', os.path.join(ROOT, 'include'), '-Wno-unused-result'
]


def _stale(obj, deps):
    if not os.path.exists(obj):
        return True
    t = os.path.getmtime(obj)
    return any(os.path.getmtime(d) > t for d in deps)


def build(verbose: bool = False, force: bool = False, single16: bool = True) -> str:
    """Build libwc_kernels.so (and, with single16, the single-piece variants libwc_kernels_single16.so and
    libwc_kernels_bf16.so); returns the first's path."""
    hdrs = [os.path.join(CSRC, h) for h in HEADERS] + [os.path.join(ROOT, 'include', 'wc_kernels.h')]
    jobs = []
    objs = []
    for src in SOURCES:
        sp = os.path.join(CSRC, src)
        obj = os.path.join(LIBDIR, 'obj', src.replace('.hip', '.o'))
        objs.append(obj)
        if force or _stale(obj, [sp] + hdrs):
            jobs.append([HIPCC] + CFLAGS + ['-c', sp, '-o', obj])
    variants = []  # (library path, objects)
    if single16:
        for tag, flag, path in (('single16', '1', SINGLE16_LIB_PATH), ('bf16', '2', BF16_LIB_PATH)):
            os.makedirs(os.path.join(LIBDIR, 'obj', tag), exist_ok=True)
            vobjs = []
            for src in SOURCES:
                if src not in SINGLE16_SOURCES:
                    vobjs.append(os.path.join(LIBDIR, 'obj', src.replace('.hip', '.o')))
                    continue
                sp = os.path.join(CSRC, src)
                obj = os.path.join(LIBDIR, 'obj', tag, src.replace('.hip', '.o'))
                vobjs.append(obj)
                if force or _stale(obj, [sp] + hdrs):
                    jobs.append([HIPCC] + CFLAGS + [f'-DWC_SINGLE16={flag}', '-c', sp, '-o', obj])
            variants.append((path, vobjs))

    def run(cmd):
        if verbose:
            print(' '.join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f'hipcc failed:\n{" ".join(cmd)}\n{r.stdout}\n{r.stderr}')
        return r

    with ThreadPoolExecutor(max_workers=min(4, max(1, len(jobs)))) as ex:
        list(ex.map(run, jobs))
    for path, lobjs in [(LIB_PATH, objs)] + variants:
        if not lobjs:
            continue
        if jobs or force or _stale(path, lobjs):
            run([HIPCC, '-shared', '-fPIC', f'--offload-arch={ARCH}', '-o', path] + lobjs)
            # A kernel whose body the host pass rejects (a device-only builtin used directly in a
            # __global__ template) loses its host stub without any diagnostic and the library then
            # fails to load: refuse to produce such a library.
            nm = subprocess.run(['nm', '-D', '--undefined-only', path], capture_output=True, text=True)
            lost = [ln.split()[-1] for ln in nm.stdout.splitlines() if '_GLOBAL__N_' in ln]
            if lost:
                os.remove(path)
                raise RuntimeError(f'{len(lost)} kernel stub(s) missing from the library, e.g. {lost[0]}')
    return LIB_PATH


if __name__ == '__main__':
    print(build(verbose='-v' in sys.argv, force='-f' in sys.argv))
