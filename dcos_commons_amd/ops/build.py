"""Builds the in-tree native artefacts for gfx950.

* ``dcos_commons_amd/ops/_amdprobe.so`` -- HIP probe kernels (C ABI, loaded with ctypes);
* ``native/build/amd-gpu-probe``       -- standalone HIP probe binary (readiness check command);
* ``native/build/amd-gpu-probed``      -- node-local readiness service (keeps the HIP runtime and the
  per-device probe contexts resident; ``amd-gpu-ready``, a CMake target, is its client);
* ``native/build/sdk-bootstrap``, ``native/build/sdk-cli`` -- C++ task bootstrap and service CLI.
* ``native/build/keytab-fix`` -- hdfs keytab rewriter run by Kerberized hdfs tasks (HADOOP-16283).
* ``native/build/sdk-agent-launcher`` -- starts and reaps the local DC/OS stand-in's task processes
  and check commands outside the master's interpreter (``mesos/containerizer.py``).

Everything is compiled directly with ``hipcc --offload-arch=gfx950`` / ``g++`` (no hipify, no
JIT cache outside the tree) so the built files travel with the repository snapshot.
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys
from typing import List

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
OPS = os.path.join(ROOT, "dcos_commons_amd", "ops")
NATIVE = os.path.join(ROOT, "native")
BUILD = os.path.join(NATIVE, "build")
BUILD_SANITIZE = os.path.join(NATIVE, "build-sanitize")  # ASan/UBSan host tools (tests only)
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950").split(";")[0] or "gfx950"


def hipcc() -> str:
    for c in (os.path.join(os.environ.get("ROCM_PATH", "/opt/rocm"), "bin", "hipcc"), shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found (ROCm toolchain required to build the gfx950 kernels)")


def _stale(out: str, srcs: List[str]) -> bool:
    if not os.path.exists(out):
        return True
    t = os.path.getmtime(out)
    return any(os.path.getmtime(s) > t for s in srcs)


def _run(cmd: List[str], verbose: bool) -> None:
    if verbose:
        print("+", " ".join(cmd), file=sys.stderr)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"build failed ({r.returncode}): {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")


def build_probe_lib(force: bool = False, verbose: bool = False) -> str:
    out = os.path.join(OPS, "_amdprobe.so")
    srcs = [os.path.join(OPS, "csrc", f) for f in ("probe_api.hip", "probe_kernels.hip")]
    if force or _stale(out, srcs):
        _run([hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared", srcs[0], "-o", out], verbose)
    return out


def build_probe_binary(force: bool = False, verbose: bool = False) -> str:
    os.makedirs(BUILD, exist_ok=True)
    out = os.path.join(BUILD, "amd-gpu-probe")
    src = os.path.join(NATIVE, "probe", "amd_gpu_probe.hip")
    deps = [src, os.path.join(OPS, "csrc", "probe_kernels.hip")]
    if force or _stale(out, deps):
        _run([hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", f"-I{os.path.join(OPS, 'csrc')}", src, "-o", out],
             verbose)
    return out


def build_probe_service(force: bool = False, verbose: bool = False) -> str:
    os.makedirs(BUILD, exist_ok=True)
    out = os.path.join(BUILD, "amd-gpu-probed")
    srcs = [os.path.join(NATIVE, "probe", "probed.cpp"), os.path.join(OPS, "csrc", "probe_api.hip")]
    deps = srcs + [os.path.join(OPS, "csrc", "probe_kernels.hip")]
    if force or _stale(out, deps):
        _run([hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-pthread", *srcs, "-o", out], verbose)
    return out


def build_cpp_tools(force: bool = False, verbose: bool = False, sanitize: bool = False) -> List[str]:
    """CMake build of the C++ natives (bootstrap, CLI, TLS crypto library) if their sources exist.

    ``sanitize=True`` builds the host tools (bootstrap, CLI, unit tests) with AddressSanitizer and
    UBSan into ``native/build-sanitize``; it is a CPU-only build, never shipped."""
    if not os.path.exists(os.path.join(NATIVE, "CMakeLists.txt")):
        return []
    out = BUILD_SANITIZE if sanitize else BUILD
    os.makedirs(out, exist_ok=True)
    names = ("sdk-bootstrap", "sdk-cli", "native-tests", "tls-tests", "amd-gpu-ready", "keytab-fix",
             "sdk-agent-launcher") + (
        () if sanitize else ("libsdktls.so",))
    targets = [os.path.join(out, n) for n in names]
    srcs = []
    for d, _, fs in os.walk(NATIVE):
        if os.path.abspath(d).startswith((os.path.abspath(BUILD), os.path.abspath(BUILD_SANITIZE))):
            continue
        srcs.extend(os.path.join(d, f) for f in fs if f.endswith((".cpp", ".h", ".hpp", ".txt")))
    if force or any(_stale(t, srcs) for t in targets):
        if sanitize:
            _run(["cmake", "-S", NATIVE, "-B", out, "-DCMAKE_BUILD_TYPE=Debug", "-DSDK_SANITIZE=ON", "-G", "Ninja"],
                 verbose)
            _run(["cmake", "--build", out, "-j", "8", "--target", *names], verbose)
        else:
            _run(["cmake", "-S", NATIVE, "-B", out, "-DCMAKE_BUILD_TYPE=Release", "-G", "Ninja"], verbose)
            _run(["cmake", "--build", out, "-j", "8"], verbose)
    return targets


def build_all(force: bool = False, verbose: bool = False) -> List[str]:
    out = [build_probe_lib(force, verbose)]
    if os.path.exists(os.path.join(NATIVE, "probe", "amd_gpu_probe.hip")):
        out.append(build_probe_binary(force, verbose))
    if os.path.exists(os.path.join(NATIVE, "probe", "probed.cpp")):
        out.append(build_probe_service(force, verbose))
    out.extend(build_cpp_tools(force, verbose))
    return out


if __name__ == "__main__":
    for p in build_all(force="--force" in sys.argv, verbose=True):
        print(p)
