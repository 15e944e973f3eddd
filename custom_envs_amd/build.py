"""Build the in-tree HIP engine library for gfx950.

    python -m custom_envs_amd.build            # -> custom_envs_amd/lib/*.so

hipcc compiles the kernels for gfx950 only (no host fallback, no other
arch); seeding.cpp is plain host C++.  The library has no torch dependency:
Python binds it with ctypes (custom_envs_amd/_native.py).
"""
import glob
import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, 'csrc')
LIBDIR = os.path.join(HERE, 'lib')
LIBNAME = 'libcustom_envs_amd.so'
DIAG_LIBNAME = 'libcustom_envs_amd_diag.so'   # -DCE_DIAG phase stamps (profiling only)
ARCH = 'gfx950'


def _hipcc():
    for cand in (os.environ.get('HIPCC'), '/opt/rocm/bin/hipcc', shutil.which('hipcc')):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError('hipcc not found; the engine requires ROCm (gfx950)')


def sources():
    return [os.path.join(CSRC, f) for f in ('engine.hip', 'optimize_mfma.hip', 'optimize_lr_persist.hip',
                                            'multi_engine.hip', 'multinn_engine.hip', 'net_engine.hip',
                                            'seeding.cpp')]


def headers():
    """Every header the sources include (all of csrc/*.h, so a new one can
    not be missed by the up-to-date check)."""
    return sorted(glob.glob(os.path.join(CSRC, '*.h'))) + [
        os.path.join(ROOT, 'include', 'custom_envs_amd.h')]


def lib_path(diag=False):
    return os.path.join(LIBDIR, DIAG_LIBNAME if diag else LIBNAME)


def up_to_date(diag=False):
    out = lib_path(diag)
    if not os.path.exists(out):
        return False
    mtime = os.path.getmtime(out)
    return all(os.path.getmtime(p) <= mtime for p in sources() + headers())


def build(force=False, verbose=False, diag=False, variant=None, defines=()):
    """Build the engine; `variant` + `defines` make an experiment build
    lib/libcustom_envs_amd_<variant>.so (selected at run time by CE_LIB)."""
    if variant:
        out = os.path.join(LIBDIR, 'libcustom_envs_amd_%s.so' % variant)
        return _compile(out, os.path.join(LIBDIR, 'obj_' + variant), list(defines), verbose)
    if not force and up_to_date(diag):
        return lib_path(diag)
    return _compile(lib_path(diag), os.path.join(LIBDIR, 'obj_diag' if diag else 'obj'),
                    ['CE_DIAG'] if diag else [], verbose)


def _compile(out, tmp, defines, verbose):
    os.makedirs(LIBDIR, exist_ok=True)
    hipcc = _hipcc()
    objs = []
    common = ['-O3', '-fPIC', '-std=c++17', '-Wall', '-I', os.path.join(ROOT, 'include')]
    common += ['-D' + d for d in defines]
    os.makedirs(tmp, exist_ok=True)
    cmds = []
    for src in sources():
        obj = os.path.join(tmp, os.path.basename(src) + '.o')
        if src.endswith('.hip'):
            cmd = [hipcc, '--offload-arch=' + ARCH, '-x', 'hip'] + common + ['-c', src, '-o', obj]
            if os.path.basename(src) in ('optimize_mfma.hip', 'optimize_lr_persist.hip') and \
                    'CE_AGPR_FORM' not in defines:
                # f64 MFMA results in VGPRs: the two-class kernel's softmax reads
                # every forward C register, and the AGPR form cost 200
                # v_accvgpr moves per wave
                cmd[-4:-4] = ['-mllvm', '-amdgpu-mfma-vgpr-form=1']
            if os.path.basename(src) == 'optimize_lr_persist.hip' and 'CE_NO_ALIGN_LOOPS' not in defines:
                # 64-byte aligned loop headers: the K-step row loop measured
                # 2.050-2.057 against 2.063-2.066 us per step (r06g)
                cmd[-4:-4] = ['-falign-loops=64']
            if os.path.basename(src) in ('optimize_mfma.hip', 'optimize_lr_persist.hip') and \
                    'CE_NO_KARG_PRELOAD' not in defines:
                # the two-class kernels' leading pointer / size arguments in
                # SGPRs at wave launch (kernarg preload, gfx950)
                cmd[-4:-4] = ['-mllvm', '-amdgpu-kernarg-preload-count=14']
        else:
            cmd = [hipcc, '-x', 'c++'] + common + ['-c', src, '-o', obj]
        if verbose:
            print(' '.join(cmd), file=sys.stderr)
        cmds.append(cmd)
        objs.append(obj)
    # one hipcc per translation unit, in parallel
    from concurrent.futures import ThreadPoolExecutor
    with ThreadPoolExecutor(max_workers=min(len(cmds), 8)) as pool:
        for proc in pool.map(lambda c: subprocess.run(c, check=True), cmds):
            pass
    # no BLAS library: every dense product is one of the engine's own MFMA kernels
    cmd = [hipcc, '--offload-arch=' + ARCH, '-shared', '-fPIC', '-o', out + '.tmp'] + objs
    subprocess.run(cmd, check=True)
    os.replace(out + '.tmp', out)
    return out


if __name__ == '__main__':
    print(build(force='--force' in sys.argv, verbose=True))
    if '--diag' in sys.argv:
        print(build(force='--force' in sys.argv, verbose=True, diag=True))
