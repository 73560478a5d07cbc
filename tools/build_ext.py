"""In-tree native build for tfk.

Compiles every ``csrc/kernels/*.hip`` with hipcc for gfx950, the pybind11 bindings with the
host compiler against torch's headers, and links ``tensorflow_k8s_amd/_C*.so``. Also builds the
C++ control plane (``cpp/``) via its Makefile. Incremental (mtime based), parallel.
No hipify, no JIT cache: the .so lives in the package directory so it travels with the repo.
"""
from __future__ import annotations

import concurrent.futures as cf
import glob
import os
import subprocess
import sys
import sysconfig

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OBJ = os.path.join(ROOT, "build", "obj")
PKG = os.path.join(ROOT, "tensorflow_k8s_amd")
ARCH = os.environ.get("TFK_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


def _torch_paths():
    import torch  # noqa: F401
    from torch.utils import cpp_extension as ce

    return ce.include_paths(device_type="cuda"), ce.library_paths(device_type="cuda")


def _stale(out: str, deps: list[str]) -> bool:
    if not os.path.exists(out):
        return True
    t = os.path.getmtime(out)
    return any(os.path.getmtime(d) > t for d in deps)


def _check_scratch(stderr: str, src: str) -> None:
    """Kernels must not spill: a scratch-using GEMM/attention kernel runs several times slower, so a
    kernel with scratch is a build ERROR (drop or retile the variant)."""
    import re
    fn = None
    bad = []
    for line in stderr.splitlines():
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            fn = m.group(1)
        m = re.search(r"ScratchSize \[bytes/lane\]: (\d+)", line)
        if m and int(m.group(1)) > 0:
            bad.append(f"{os.path.basename(src)}: {fn} uses {m.group(1)} B/lane of scratch")
    if bad:
        raise RuntimeError("kernels spill to scratch:\n  " + "\n  ".join(bad))


def _run(cmd: list[str]) -> None:
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        sys.stderr.write(r.stdout + r.stderr)
        raise RuntimeError("build failed: " + " ".join(cmd[:3]) + " ... " + cmd[-1])
    if "-Rpass-analysis=kernel-resource-usage" in cmd:
        try:
            _check_scratch(r.stderr, cmd[-3])
        except RuntimeError:
            os.remove(cmd[-1])  # keep the spilling object from looking up to date
            raise


def _extra_flags(src: str) -> list[str]:
    """Per-file hipcc flags from a `// hipcc-flags: ...` line in the first lines of a .hip source
    (e.g. a scheduler strategy for one GEMM variant)."""
    with open(src) as f:
        for _ in range(5):
            line = f.readline()
            if line.startswith("// hipcc-flags:"):
                return line.split(":", 1)[1].split()
    return []


def ext_path() -> str:
    return os.path.join(PKG, "_C" + sysconfig.get_config_var("EXT_SUFFIX"))


def build_kernels(jobs: int | None = None, verbose: bool = False) -> str:
    headers = glob.glob(os.path.join(ROOT, "csrc", "kernels", "*.h"))
    srcs = (glob.glob(os.path.join(ROOT, "csrc", "kernels", "*.hip")) + glob.glob(os.path.join(ROOT, "csrc", "bindings", "*.cpp"))
            + headers + glob.glob(os.path.join(ROOT, "cpp", "*", "*.h"))
            + [os.path.join(ROOT, r) for r in ("cpp/runtime/tfbundle.cc", "cpp/common/util.cc", "cpp/common/json.cc")])
    so = ext_path()
    if os.path.exists(so) and not _stale(so, srcs):
        # up to date -- also the case on a GPU box, whose snapshot carries the .so but not build/obj
        if verbose:
            print(f"[tfk build] {so} is up to date")
        return so
    os.makedirs(OBJ, exist_ok=True)
    inc, libs = _torch_paths()
    jobs = jobs or min(16, os.cpu_count() or 4)
    tasks = []
    objs = []
    for src in sorted(glob.glob(os.path.join(ROOT, "csrc", "kernels", "*.hip"))):
        out = os.path.join(OBJ, os.path.basename(src) + ".o")
        objs.append(out)
        if _stale(out, [src] + headers):
            tasks.append([HIPCC, "-c", "-fPIC", "-O3", "-std=c++17", f"--offload-arch={ARCH}",
                          "-munsafe-fp-atomics"] + _extra_flags(src) + ["-Rpass-analysis=kernel-resource-usage", src, "-o", out])
    py_inc = sysconfig.get_paths()["include"]
    cpp_hdrs = glob.glob(os.path.join(ROOT, "cpp", "*", "*.h"))
    for src in sorted(glob.glob(os.path.join(ROOT, "csrc", "bindings", "*.cpp"))):
        out = os.path.join(OBJ, os.path.basename(src) + ".o")
        objs.append(out)
        if _stale(out, [src] + headers + cpp_hdrs):
            cmd = ["g++", "-c", "-fPIC", "-O2", "-std=c++17", "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1",
                   "-D_GLIBCXX_USE_CXX11_ABI=1", "-DTORCH_EXTENSION_NAME=_C", "-DTORCH_API_INCLUDE_EXTENSION_H",
                   f"-I{py_inc}"] + [f"-I{p}" for p in inc] + [src, "-o", out]
            tasks.append(cmd)
    # native checkpoint (TF bundle) + its deps from the control-plane tree, linked into _C
    for rel in ("cpp/runtime/tfbundle.cc", "cpp/common/util.cc", "cpp/common/json.cc"):
        src = os.path.join(ROOT, rel)
        out = os.path.join(OBJ, "cp_" + os.path.basename(src) + ".o")
        objs.append(out)
        if _stale(out, [src] + cpp_hdrs):
            tasks.append(["g++", "-c", "-fPIC", "-O2", "-std=c++17", "-pthread", src, "-o", out])
    if tasks:
        with cf.ThreadPoolExecutor(jobs) as ex:
            for f in [ex.submit(_run, t) for t in tasks]:
                f.result()
    so = ext_path()
    if tasks or _stale(so, objs):
        tlib = [p for p in libs if "torch" in p][0]
        cmd = ["g++", "-shared", "-o", so] + objs + [f"-L{tlib}", "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu",
                                                     "-ltorch_hip", "-ltorch_python", "-lamdhip64",
                                                     # torch's own librccl.so (SONAME librccl.so.1): one RCCL
                                                     # instance in the process, shared with torch.distributed
                                                     "-lrccl",
                                                     f"-Wl,-rpath,{tlib}"]
        _run(cmd)
    if verbose:
        print(f"[tfk build] {len(tasks)} objects rebuilt -> {so}")
    return so


def build_control_plane(jobs: int | None = None, verbose: bool = False) -> None:
    mk = os.path.join(ROOT, "cpp", "Makefile")
    if not os.path.exists(mk):
        return
    jobs = jobs or min(16, os.cpu_count() or 4)
    r = subprocess.run(["make", "-C", os.path.join(ROOT, "cpp"), f"-j{jobs}"], capture_output=True, text=True)
    if r.returncode != 0:
        sys.stderr.write(r.stdout[-4000:] + r.stderr[-8000:])
        raise RuntimeError("control-plane build failed")
    if verbose:
        print("[tfk build] control plane ok")


def build_all(verbose: bool = True) -> None:
    build_kernels(verbose=verbose)
    build_control_plane(verbose=verbose)


if __name__ == "__main__":
    build_all()
