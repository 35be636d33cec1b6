"""In-tree build of the native extension ``django_assistant_bot_amd/_native*.so``.

Every ``csrc/kernels/*.hip`` file is compiled by ``hipcc --offload-arch=gfx950`` (CDNA4 only, no
hipify, no CUDA path), the host runtime ``csrc/runtime/*.cpp`` and the pybind11 bindings are
compiled by hipcc as host C++, and everything is linked into one shared object next to this file
(so it travels with the repository snapshot to the GPU box).  Objects are rebuilt only when a
source or header is newer than the object.

    python -m django_assistant_bot_amd.build [--force] [-j N] [--debug]
    python -m django_assistant_bot_amd.build --selftest asan|tsan   # host runtime under sanitizers
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import subprocess
import sys
import sysconfig
from pathlib import Path

PKG = Path(__file__).resolve().parent
CSRC = PKG / "csrc"
BUILD = PKG / "_build"
ARCH = os.environ.get("DAB_OFFLOAD_ARCH", "gfx950")


def _hipcc() -> str:
    rocm = os.environ.get("ROCM_PATH", "/opt/rocm")
    cand = Path(rocm) / "bin" / "hipcc"
    return str(cand) if cand.exists() else "hipcc"


def ext_path() -> Path:
    suffix = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
    return PKG / f"_native{suffix}"


def _headers() -> list[Path]:
    return sorted(CSRC.rglob("*.h"))


def _needs(obj: Path, src: Path, deps: list[Path]) -> bool:
    if not obj.exists():
        return True
    t = obj.stat().st_mtime
    return src.stat().st_mtime > t or any(d.stat().st_mtime > t for d in deps)


def _compile(cmd: list[str]) -> tuple[list[str], int, str]:
    p = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    return cmd, p.returncode, p.stdout


# Kernels allowed a scratch (stack) frame: stream_gemm tuning configurations that no model path
# launches (cfg 14-16, 24, 26: benchmarks/decode_ab.py only).  Anything else with a frame is a build
# error -- a runtime-indexed register array the compiler moved to memory (a fully unrolled
# epilogue that stopped unrolling put gemm256's accumulators there in round 4: 3x slower).
_SCRATCH_OK = ("stream_gemm_kernelILi8ELi2ELi1ELi128ELi4ELi4ELi4E", "stream_gemm_kernelILi8ELi2ELi1ELi128ELi4ELi4ELi2E",
               "stream_gemm_kernelILi4ELi2ELi1ELi128ELi4ELi6ELi4E", "stream_gemm_kernelILi16ELi1ELi1ELi128ELi2ELi3ELi1E",
               "stream_gemm_kernelILi16ELi2ELi1ELi128ELi2ELi2ELi2E")


def scratch_kernels(log: str) -> list[tuple[str, int]]:
    """(kernel, bytes per lane) of every kernel with a scratch frame in a
    ``-Rpass-analysis=kernel-resource-usage`` compile log."""
    out, name = [], None
    for line in log.splitlines():
        if "Function Name:" in line:
            name = line.split("Function Name:", 1)[1].split()[0]
        elif "ScratchSize [bytes/lane]:" in line and name:
            n = int(line.split("ScratchSize [bytes/lane]:", 1)[1].split()[0])
            if n:
                out.append((name, n))
    return out


def build(force: bool = False, jobs: int | None = None, debug: bool = False, verbose: bool = False) -> Path:
    import pybind11

    BUILD.mkdir(exist_ok=True)
    hipcc = _hipcc()
    opt = ["-O0", "-g"] if debug else ["-O3"]
    common = ["-std=c++17", "-fPIC", *opt, f"-I{CSRC}", "-Wno-unused-result", "-Wno-unused-command-line-argument"]
    py_inc = [f"-I{sysconfig.get_paths()['include']}", f"-I{pybind11.get_include()}"]
    deps = _headers()
    jobs_list: list[tuple[list[str], Path]] = []
    objs: list[Path] = []
    for src in sorted((CSRC / "kernels").glob("*.hip")):
        obj = BUILD / (src.stem + ".hip.o")
        objs.append(obj)
        if force or _needs(obj, src, deps):
            jobs_list.append(([hipcc, f"--offload-arch={ARCH}", *common, "-Rpass-analysis=kernel-resource-usage", "-c",
                               str(src), "-o", str(obj)], obj))
    host_srcs = sorted((CSRC / "runtime").glob("*.cpp")) + [CSRC / "bindings.cpp"]
    for src in host_srcs:
        obj = BUILD / (src.stem + ".cpp.o")
        objs.append(obj)
        if force or _needs(obj, src, deps):
            jobs_list.append(([hipcc, *common, *py_inc, "-fvisibility=hidden", "-c", str(src), "-o", str(obj)], obj))
    out = ext_path()
    n = jobs or min(16, os.cpu_count() or 4)
    failed = []
    with cf.ThreadPoolExecutor(max_workers=n) as ex:
        for cmd, rc, log in ex.map(lambda j: _compile(j[0]), jobs_list):
            if verbose or rc:
                print(" ".join(cmd), file=sys.stderr)
                print(log, file=sys.stderr)
            if rc:
                failed.append(cmd[-1])
            bad = [(k, b) for k, b in scratch_kernels(log) if not any(a in k for a in _SCRATCH_OK)]
            if bad and not debug:
                Path(cmd[-1]).unlink(missing_ok=True)  # rebuilt (and re-checked) next time
                raise RuntimeError(f"kernels with a scratch frame (runtime-indexed registers): {bad}")
    if failed:
        raise RuntimeError(f"native build failed for: {failed}")
    if force or jobs_list or not out.exists():
        link = [hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", *[str(o) for o in objs], "-o", str(out), "-lpthread", "-ldl"]
        cmd, rc, log = _compile(link)
        if rc:
            print(" ".join(cmd), file=sys.stderr)
            print(log, file=sys.stderr)
            raise RuntimeError("native link failed")
    return out


SANITIZERS = {"asan": ["-fsanitize=address,undefined", "-fno-omit-frame-pointer", "-fno-sanitize-recover=undefined"],
              "tsan": ["-fsanitize=thread"]}


def selftest(kind: str = "asan", out_dir: Path | None = None) -> tuple[int, str]:
    """Compiles csrc/tests/runtime_selftest.cpp with the host runtime sources (plain g++, no HIP:
    GPU sanitizers are not available on this hardware pool) under ASan+UBSan or TSan, runs it and
    returns (exit code, output)."""
    out_dir = out_dir or BUILD
    out_dir.mkdir(exist_ok=True)
    exe = out_dir / f"runtime_selftest_{kind}"
    srcs = [CSRC / "tests" / "runtime_selftest.cpp", *sorted((CSRC / "runtime").glob("*.cpp"))]
    cmd = ["g++", "-std=c++17", "-g", "-O1", *SANITIZERS[kind], f"-I{CSRC}", *map(str, srcs), "-o", str(exe),
           "-ldl", "-lpthread"]
    _, rc, log = _compile(cmd)
    if rc:
        return rc, log
    p = subprocess.run([str(exe)], stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=600)
    return p.returncode, p.stdout


def main() -> None:
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", "--jobs", type=int, default=None)
    ap.add_argument("--debug", action="store_true")
    ap.add_argument("-v", "--verbose", action="store_true")
    ap.add_argument("--selftest", choices=sorted(SANITIZERS), default=None)
    a = ap.parse_args()
    if a.selftest:
        rc, log = selftest(a.selftest)
        print(log)
        sys.exit(rc)
    print(build(force=a.force, jobs=a.jobs, debug=a.debug, verbose=a.verbose))


if __name__ == "__main__":
    main()
