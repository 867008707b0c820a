"""Build librdl_hip.so (HIP, gfx950), libradler_amd.so (host C++) and the
`radler` pybind11 module in-tree. Incremental: objects are rebuilt when their
source or any header in csrc/ or include/ is newer.

    python ska-sdp-func-radler_amd/build.py [-j N] [--clean]
"""
import argparse
import concurrent.futures as cf
import glob
import os
import shutil
import subprocess
import sys
import sysconfig

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
INCLUDE = os.path.join(ROOT, "include")
CSRC = os.path.join(PKG, "csrc")
BUILD = os.path.join(PKG, "build")
LIB = os.path.join(PKG, "lib")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
ARCH = os.environ.get("RDL_OFFLOAD_ARCH", "gfx950")

HIPCC = os.path.join(ROCM, "bin", "hipcc")
HIP_FLAGS = ["-O3", "-std=c++17", f"--offload-arch={ARCH}", "-fPIC",
             "-ffp-contract=off", "-Wall", "-Wno-unused-function",
             f"-I{INCLUDE}", f"-I{os.path.join(CSRC, 'hip')}"]
CXX = os.environ.get("CXX", "g++")
# Host code: the reference builds with -O3 (cpp/CMakeLists.txt:73). Host-side
# float math that must match the reference bit-for-bit (scale kernels,
# thresholds) is written with explicit std::fma where GCC contracts.
CXX_FLAGS = ["-O2", "-std=c++17", "-fPIC", "-ffp-contract=off", "-Wall",
             "-pthread", f"-I{INCLUDE}", f"-I{os.path.join(CSRC, 'host')}",
             # logpoly.h: the log-polynomial fitter shared by kernels and host
             f"-I{os.path.join(CSRC, 'hip')}"]


def newest_header():
    hs = glob.glob(os.path.join(CSRC, "**", "*.h"), recursive=True)
    hs += glob.glob(os.path.join(INCLUDE, "*.h"))
    return max((os.path.getmtime(h) for h in hs), default=0.0)


def stale(out, srcs, hdr_time):
    if not os.path.exists(out):
        return True
    t = os.path.getmtime(out)
    return any(os.path.getmtime(s) > t for s in srcs) or hdr_time > t


def run(cmd):
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError("build failed:\n" + " ".join(cmd) + "\n" + r.stdout + r.stderr)
    return r


def compile_all(jobs, items):
    errors = []
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        futs = {ex.submit(run, cmd): out for out, cmd in items}
        for f in cf.as_completed(futs):
            try:
                f.result()
            except Exception as e:  # noqa: BLE001
                errors.append(str(e))
    if errors:
        raise RuntimeError("\n".join(errors))


def link(cmd_prefix, out, rest):
    """Link to a temporary name, then rename over `out` (atomic): a copy of the
    tree taken while a build runs never holds a half-written library."""
    tmp = out + ".tmp"
    run([*cmd_prefix, "-o", tmp, *rest])
    os.replace(tmp, out)


def build(jobs=8, verbose=False):
    os.makedirs(BUILD, exist_ok=True)
    os.makedirs(LIB, exist_ok=True)
    hdr = newest_header()

    # ---- librdl_hip.so
    hip_srcs = sorted(glob.glob(os.path.join(CSRC, "hip", "*.hip")))
    hip_objs, items = [], []
    for src in hip_srcs:
        obj = os.path.join(BUILD, "hip_" + os.path.basename(src) + ".o")
        hip_objs.append(obj)
        if stale(obj, [src], hdr):
            items.append((obj, [HIPCC, *HIP_FLAGS, "-c", src, "-o", obj]))
    compile_all(jobs, items)
    hip_so = os.path.join(LIB, "librdl_hip.so")
    if items or not os.path.exists(hip_so):
        link([HIPCC, "-shared", f"--offload-arch={ARCH}"], hip_so,
             [*hip_objs, f"-L{ROCM}/lib", "-lrocfft", "-lrccl", f"-Wl,-rpath,{ROCM}/lib"])

    # ---- libradler_amd.so (host C++ mirror of the radler API)
    host_srcs = sorted(glob.glob(os.path.join(CSRC, "host", "*.cc")))
    host_objs, items = [], []
    for src in host_srcs:
        obj = os.path.join(BUILD, "host_" + os.path.basename(src) + ".o")
        host_objs.append(obj)
        if stale(obj, [src], hdr):
            items.append((obj, [CXX, *CXX_FLAGS, "-c", src, "-o", obj]))
    compile_all(jobs, items)
    host_so = os.path.join(LIB, "libradler_amd.so")
    if host_objs and (items or stale(host_so, [hip_so], 0.0)):
        link([CXX, "-shared", "-pthread"], host_so,
             [*host_objs, f"-L{LIB}", "-lrdl_hip", "-Wl,-rpath,$ORIGIN"])

    # ---- radler pybind11 module
    py_srcs = sorted(glob.glob(os.path.join(CSRC, "python", "*.cc")))
    if py_srcs:
        import pybind11
        ext = sysconfig.get_config_var("EXT_SUFFIX")
        mod = os.path.join(PKG, "radler" + ext)
        py_flags = [*CXX_FLAGS, f"-I{pybind11.get_include()}",
                    f"-I{sysconfig.get_paths()['include']}", "-fvisibility=hidden"]
        py_objs, items = [], []
        for src in py_srcs:
            obj = os.path.join(BUILD, "py_" + os.path.basename(src) + ".o")
            py_objs.append(obj)
            if stale(obj, [src], hdr):
                items.append((obj, [CXX, *py_flags, "-c", src, "-o", obj]))
        compile_all(jobs, items)
        if items or stale(mod, [host_so], 0.0):
            link([CXX, "-shared", "-pthread"], mod,
                 [*py_objs, f"-L{LIB}", "-lradler_amd", "-lrdl_hip", "-Wl,-rpath,$ORIGIN/lib"])
    return hip_so


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("-j", type=int, default=min(8, os.cpu_count() or 8))
    ap.add_argument("--clean", action="store_true")
    args = ap.parse_args()
    if args.clean:
        shutil.rmtree(BUILD, ignore_errors=True)
        shutil.rmtree(LIB, ignore_errors=True)
    print(build(args.j))


if __name__ == "__main__":
    sys.exit(main())
