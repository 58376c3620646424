"""Build libtpe_hip.so in-tree for gfx950:  python -m hyperopt_amd.build"""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, 'csrc', 'tpe_kernels.hip')
OUT = os.path.join(HERE, 'libtpe_hip.so')
ARCH = os.environ.get('TPE_OFFLOAD_ARCH', 'gfx950')


def build(force=False, verbose=False):
    if (not force and os.path.exists(OUT) and os.path.getmtime(OUT) >= os.path.getmtime(SRC)
            and os.path.getmtime(OUT) >= os.path.getmtime(os.path.join(HERE, '..', 'include', 'tpe_hip.h'))):
        return OUT
    hipcc = os.environ.get('HIPCC', '/opt/rocm/bin/hipcc')
    cmd = [hipcc, '-O3', '--offload-arch=' + ARCH, '-std=c++17', '-shared', '-fPIC',
           '-Wall', '-Wno-unused-command-line-argument', '-o', OUT + '.tmp', SRC]
    if verbose:
        print(' '.join(cmd))
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        sys.stderr.write(r.stdout + r.stderr)
        raise RuntimeError('hipcc failed for %s' % SRC)
    os.replace(OUT + '.tmp', OUT)
    return OUT


if __name__ == '__main__':
    print(build(force='--force' in sys.argv, verbose=True))
