"""Build libtpe_hip.so in-tree for gfx950:  python -m hyperopt_amd.build"""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, 'csrc', 'tpe_kernels.hip')
HOST_SRC = os.path.join(HERE, 'csrc', 'tpe_host.cpp')
SUGGEST_SRC = os.path.join(HERE, 'csrc', 'tpe_suggest.cpp')
POOL_SRC = os.path.join(HERE, 'csrc', 'tpe_pool.cpp')
OUT = os.path.join(HERE, 'libtpe_hip.so')
ARCH = os.environ.get('TPE_OFFLOAD_ARCH', 'gfx950')
# host ISA baseline of the runtime (any x86-64 host); the vectorised pack loops
# carry their own AVX2 clones (target_clones), picked at load time
HOST_MARCH = os.environ.get('TPE_HOST_MARCH', 'x86-64-v2')


def build(force=False, verbose=False, out=OUT, defines=()):
    """hipcc the kernels, g++ the host runtime (-ffp-contract=off: numpy float64
    semantics), link both into hyperopt_amd/libtpe_hip.so (or `out`, with extra
    -D `defines` on the kernels: A/B variants for tools/)."""
    OUT = out
    deps = [SRC, HOST_SRC, SUGGEST_SRC, POOL_SRC, os.path.join(HERE, 'csrc', 'tpe_pool.h'), os.path.join(HERE, 'csrc', 'sort_net.h'),
            os.path.join(HERE, '..', 'include', 'tpe_hip.h'), os.path.abspath(__file__)]
    if out == os.path.join(HERE, 'libtpe_hip.so'):
        build_hostaddr(force, verbose)
    if not force and os.path.exists(OUT) and all(os.path.getmtime(OUT) >= os.path.getmtime(d) for d in deps):
        return OUT
    hipcc = os.environ.get('HIPCC', '/opt/rocm/bin/hipcc')
    gxx = os.environ.get('CXX', 'g++')
    tmp = OUT + '.tmp'
    tag = os.path.splitext(os.path.basename(OUT))[0]
    host_o = os.path.join(HERE, 'csrc', 'tpe_host.o')
    suggest_o = os.path.join(HERE, 'csrc', 'tpe_suggest.o')
    pool_o = os.path.join(HERE, 'csrc', 'tpe_pool.o')
    dev_o = os.path.join(HERE, 'csrc', 'tpe_kernels.o' if not defines else tag + '.o')
    hdr = [os.path.join(HERE, '..', 'include', 'tpe_hip.h'), os.path.join(HERE, 'csrc', 'tpe_pool.h'),
           os.path.join(HERE, 'csrc', 'sort_net.h')]
    host_flags = [gxx, '-O3', '-march=' + HOST_MARCH, '-std=c++17', '-fPIC', '-Wall']
    numpy_fp = ['-ffp-contract=off', '-fno-fast-math', '-fno-trapping-math']
    # (object, its sources, compile command): an object is rebuilt when a source
    # is newer than it (force: always)
    objs = [
        (host_o, [HOST_SRC] + hdr, host_flags + numpy_fp + ['-c', HOST_SRC, '-o', host_o]),
        (suggest_o, [SUGGEST_SRC] + hdr, host_flags + numpy_fp + ['-c', SUGGEST_SRC, '-o', suggest_o]),
        (pool_o, [POOL_SRC] + hdr, host_flags + ['-pthread', '-c', POOL_SRC, '-o', pool_o]),
        (dev_o, [SRC] + hdr, [hipcc, '-O3', '--offload-arch=' + ARCH, '-std=c++17', '-fPIC', '-Wall',
                              '-Wno-unused-command-line-argument'] + ['-D' + d for d in defines] +
         ['-c', SRC, '-o', dev_o]),
    ]
    cmds = [c for o, srcs, c in objs
            if force or not os.path.exists(o) or any(os.path.getmtime(s) > os.path.getmtime(o) for s in srcs)]
    cmds.append([hipcc, '-shared', '-fPIC', '--offload-arch=' + ARCH, '-Wno-unused-command-line-argument', '-o', tmp,
                 dev_o, host_o, suggest_o, pool_o, '-pthread'])
    for cmd in cmds:
        if verbose:
            print(' '.join(cmd))
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            sys.stderr.write(r.stdout + r.stderr)
            raise RuntimeError('build step failed: %s' % cmd[0])
    os.replace(tmp, OUT)
    return OUT


def build_hostaddr(force=False, verbose=False):
    """gcc the _hostaddr CPython module (csrc/hostaddr.c) in-tree."""
    import sysconfig
    import numpy
    src = os.path.join(HERE, 'csrc', 'hostaddr.c')
    out = os.path.join(HERE, '_hostaddr' + sysconfig.get_config_var('EXT_SUFFIX'))
    if not force and os.path.exists(out) and os.path.getmtime(out) >= os.path.getmtime(src):
        return out
    cmd = [os.environ.get('CC', 'gcc'), '-O2', '-shared', '-fPIC', '-Wall', '-I', sysconfig.get_paths()['include'],
           '-I', numpy.get_include(), src, '-o', out + '.tmp']
    if verbose:
        print(' '.join(cmd))
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        sys.stderr.write(r.stdout + r.stderr)
        raise RuntimeError('build step failed: %s' % cmd[0])
    os.replace(out + '.tmp', out)
    return out


if __name__ == '__main__':
    print(build(force='--force' in sys.argv, verbose=True))
