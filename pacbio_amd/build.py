"""Build recipe for the MI355X-native jf_aligner path (no cmake/ninja needed).

Products (in-tree, git-ignored, shipped to the GPU box by gpurun):
  pacbio_amd/libpbgpu.so     HIP kernels + C ABI (include/pbgpu.h), gfx950 only
  pacbio_amd/bin/jf_aligner  drop-in CLI over the C ABI
Test infrastructure (never linked into the products):
  oracle/liboracle.so, oracle/pb_oracle   CPU restatement (parity oracle)
  oracle/_ref/*                           reference-source harnesses (only
                                          when /root/reference is present)
  tools/libpbsynth.so, tools/pbsynth      synthetic workload generator
"""
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "pacbio_amd")
CSRC = os.path.join(PKG, "csrc")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"
HIPFLAGS = ["-O3", f"--offload-arch={ARCH}", "-std=c++17", "-fPIC", "-ffp-contract=off",
            "-Wno-unused-result", "-I" + os.path.join(ROOT, "include")]


def _run(cmd, cwd=None):
    r = subprocess.run(cmd, cwd=cwd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        sys.stderr.write(r.stdout)
        raise RuntimeError("build step failed: " + " ".join(cmd))
    return r.stdout


def _newer(out, srcs):
    if not os.path.exists(out):
        return True
    t = os.path.getmtime(out)
    return any(os.path.getmtime(s) > t for s in srcs)


def build_pbgpu(force=False):
    objdir = os.path.join(ROOT, "build")
    os.makedirs(objdir, exist_ok=True)
    hdrs = [os.path.join(CSRC, h) for h in ("pbgpu_internal.h", "pbgpu_host.h", "pbgpu_fmt.h")] + \
        [os.path.join(ROOT, "include", "pbgpu.h")]
    srcs = ["pbgpu_kernels.hip", "pbgpu_api.hip", "pbgpu_format.hip", "pbgpu_run.hip"]
    objs = []
    jobs = []
    for s in srcs:
        src = os.path.join(CSRC, s)
        obj = os.path.join(objdir, s + ".o")
        objs.append(obj)
        if force or _newer(obj, [src] + hdrs):
            jobs.append([HIPCC] + HIPFLAGS + ["-c", src, "-o", obj])
    with ThreadPoolExecutor(len(jobs) or 1) as ex:
        list(ex.map(_run, jobs))
    lib = os.path.join(PKG, "libpbgpu.so")
    if force or jobs or _newer(lib, objs):
        _run([HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", lib] + objs +
             ["-Wl,-soname,libpbgpu.so", "-L/opt/rocm/lib", "-lrccl", "-Wl,-rpath,/opt/rocm/lib", "-lz", "-lpthread"])
    bindir = os.path.join(PKG, "bin")
    os.makedirs(bindir, exist_ok=True)
    cli = os.path.join(bindir, "jf_aligner")
    cli_src = os.path.join(CSRC, "jf_aligner.cpp")
    if force or _newer(cli, [cli_src, lib] + hdrs):
        _run(["g++", "-O2", "-std=c++17", "-o", cli, cli_src, "-I" + os.path.join(ROOT, "include"),
              "-L" + PKG, "-lpbgpu", "-Wl,-rpath,$ORIGIN/..", "-lpthread"])
    # create_mega_reads: the same library + the host overlap graph (no FMA contraction:
    # its double arithmetic follows overlap_graph.cc's operation order)
    cmr = os.path.join(bindir, "create_mega_reads")
    cmr_src = [os.path.join(CSRC, f) for f in ("create_mega_reads.cpp", "overlap_graph.cpp")]
    if force or _newer(cmr, cmr_src + [os.path.join(CSRC, "overlap_graph.hpp"), lib] + hdrs):
        _run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-o", cmr] + cmr_src +
             ["-I" + os.path.join(ROOT, "include"), "-L" + PKG, "-lpbgpu", "-Wl,-rpath,$ORIGIN/..", "-lpthread"])
    return lib


def build_pbgpu_variant(name, defines, kernels_only=False):
    """Experiment / profiling variant libpbgpu_<name>.so built with extra -D
    flags (tools/prof_*.py, tools/exp_*.py); never the product library.
    kernels_only: the defines touch pbgpu_kernels.hip alone, the other objects
    are the product's (build_pbgpu first)."""
    objdir = os.path.join(ROOT, "build", name)
    os.makedirs(objdir, exist_ok=True)
    jobs, objs = [], []
    if kernels_only:
        build_pbgpu()
    for s in ["pbgpu_kernels.hip", "pbgpu_api.hip", "pbgpu_format.hip", "pbgpu_run.hip"]:
        if kernels_only and s != "pbgpu_kernels.hip":
            objs.append(os.path.join(ROOT, "build", s + ".o"))
            continue
        obj = os.path.join(objdir, s + ".o")
        jobs.append([HIPCC] + HIPFLAGS + list(defines) + ["-c", os.path.join(CSRC, s), "-o", obj])
        objs.append(obj)
    with ThreadPoolExecutor(len(jobs)) as ex:
        list(ex.map(_run, jobs))
    lib = os.path.join(PKG, f"libpbgpu_{name}.so")
    _run([HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", lib] + objs +
         ["-L/opt/rocm/lib", "-lrccl", "-Wl,-rpath,/opt/rocm/lib", "-lz", "-lpthread"])
    return lib


def build_pbgpu_prof():
    """Phase-profiling variant (-DPBGPU_PROF) for tools/prof_lis.py; never the product library."""
    return build_pbgpu_variant("prof", ["-DPBGPU_PROF"])


def build_oracle():
    odir = os.path.join(ROOT, "oracle")
    _run(["make", "-s", "-j8", "-C", odir, "all"])
    if os.path.isdir("/root/reference"):
        _run(["make", "-s", "-j8", "-C", odir, "ref"])


def build_tools():
    tdir = os.path.join(ROOT, "tools")
    src = os.path.join(tdir, "pbsynth.cc")
    lib = os.path.join(tdir, "libpbsynth.so")
    if _newer(lib, [src]):
        _run(["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-o", lib, src, "-pthread"])
    exe = os.path.join(tdir, "pbsynth")
    if _newer(exe, [src]):
        _run(["g++", "-O2", "-std=c++17", "-DPBSYNTH_MAIN", "-o", exe, src, "-pthread"])


def build_all(force=False):
    with ThreadPoolExecutor(3) as ex:
        f1 = ex.submit(build_pbgpu, force)
        f2 = ex.submit(build_oracle)
        f3 = ex.submit(build_tools)
        f1.result(); f2.result(); f3.result()


if __name__ == "__main__":
    build_all(force="--force" in sys.argv)
    print("ok")
