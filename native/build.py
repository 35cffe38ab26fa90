"""Builds the native components in-tree (no pip install, no JIT cache).

Outputs (git-ignored, but shipped to the GPU box by gpurun):
  nanogpu/_native<EXT>   C++17 core: ledger, policies, topology reader (g++ / pybind11)
  nanogpu/_probe<EXT>    HIP probe kernels for gfx950 (hipcc --offload-arch=gfx950)
  native/bin/nanogpu-topo   standalone topology CLI (node agent without Python)

Usage: python native/build.py [--force] [--no-hip] [--sanitize address|thread|undefined]
"""
from __future__ import annotations

import argparse
import hashlib
import os
import shutil
import subprocess
import sys
import sysconfig
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
NATIVE = ROOT / "native"
PKG = ROOT / "nanogpu"
BUILD = NATIVE / "build"
ROCM = Path(os.environ.get("ROCM_PATH", "/opt/rocm"))
EXT = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
ARCH = os.environ.get("NANOGPU_OFFLOAD_ARCH", "gfx950")

CORE_SOURCES = ["alloc.cpp", "ledger.cpp", "topo.cpp", "json.cpp", "frontend.cpp", "schedsim.cpp", "apiserver.cpp",
                "kubewriter.cpp", "kubewriter_evented.cpp", "podwatch.cpp", "sampler.cpp"]


def _pybind_includes() -> list[str]:
    import pybind11

    return [f"-I{pybind11.get_include()}", f"-I{sysconfig.get_paths()['include']}"]


def _digest(deps: list[Path], flags: list[str]) -> str:
    h = hashlib.sha256("\0".join(flags).encode())
    for d in sorted(deps):
        h.update(str(d.relative_to(ROOT) if d.is_relative_to(ROOT) else d).encode())
        h.update(d.read_bytes())
    return h.hexdigest()


def _stamp(out: Path) -> Path:
    return out.with_name(out.name + ".sha256")


def _fresh(out: Path, deps: list[Path], flags: list[str]) -> bool:
    """`out` was built from exactly these sources and flags (a content hash, not mtimes: a
    copied tree or a checkout keeps stale binaries' mtimes newer than changed sources)."""
    st = _stamp(out)
    return out.exists() and st.exists() and st.read_text().strip() == _digest(deps, flags)


def _done(out: Path, deps: list[Path], flags: list[str]) -> Path:
    _stamp(out).write_text(_digest(deps, flags) + "\n")
    return out


def _run(cmd: list[str]) -> None:
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        sys.stderr.write(" ".join(cmd) + "\n" + r.stdout + r.stderr)
        raise RuntimeError(f"native build failed: {cmd[0]} exited {r.returncode}")


def _headers() -> list[Path]:
    return sorted((NATIVE / "include").rglob("*.h"))


def build_core(force: bool = False, sanitize: str | None = None) -> Path:
    out = PKG / f"_native{EXT}"
    srcs = [NATIVE / "src" / s for s in CORE_SOURCES] + [NATIVE / "src" / "bindings.cpp"]
    if sanitize:
        out = BUILD / f"san-{sanitize}" / "nanogpu" / f"_native{EXT}"
    deps = srcs + _headers() + [Path(__file__)]
    if not force and _fresh(out, deps, [sanitize or ""]):
        return out
    objdir = BUILD / (f"san-{sanitize}" if sanitize else "obj")
    objdir.mkdir(parents=True, exist_ok=True)
    out.parent.mkdir(parents=True, exist_ok=True)
    flags = ["-std=c++17", "-fPIC", "-fvisibility=hidden", "-Wall", "-Wextra", "-Wno-unused-parameter",
             f"-I{NATIVE / 'include'}", f"-I{ROCM / 'include'}"] + _pybind_includes()
    if sanitize:
        flags += ["-O1", "-g", "-fno-omit-frame-pointer", f"-fsanitize={sanitize}"]
    else:
        flags += ["-O3", "-g1", "-DNDEBUG"]

    def compile_one(src: Path) -> Path:
        obj = objdir / (src.stem + ".o")
        _run(["g++", *flags, "-c", str(src), "-o", str(obj)])
        return obj

    with ThreadPoolExecutor(max_workers=min(4, os.cpu_count() or 1)) as ex:
        objs = list(ex.map(compile_one, srcs))
    link = ["g++", "-shared", *[str(o) for o in objs], "-o", str(out), "-ldl", "-lpthread", "-lssl", "-lcrypto"]
    if sanitize:
        link.append(f"-fsanitize={sanitize}")
    _run(link)
    return _done(out, deps, [sanitize or ""])


def build_topo_cli(force: bool = False) -> Path:
    out = NATIVE / "bin" / "nanogpu-topo"
    srcs = [NATIVE / "src" / "topo.cpp", NATIVE / "tools" / "topo_main.cpp"]
    deps = srcs + _headers() + [Path(__file__)]
    if not force and _fresh(out, deps, []):
        return out
    out.parent.mkdir(parents=True, exist_ok=True)
    _run(["g++", "-std=c++17", "-O2", f"-I{NATIVE / 'include'}", f"-I{ROCM / 'include'}",
          *[str(s) for s in srcs], "-o", str(out), "-ldl"])
    return _done(out, deps, [])


SANITIZERS = {"plain": [], "asan": ["-fsanitize=address,undefined", "-fno-sanitize-recover=undefined"],
              "tsan": ["-fsanitize=thread"]}


def build_stress(kind: str = "plain", force: bool = False) -> Path:
    """Host-only stress driver (native/tests/stress_main.cpp) linked against the core
    sources, optionally under ASan+UBSan or TSan (no GPU code involved)."""
    out = NATIVE / "bin" / f"nanogpu-stress-{kind}"
    srcs = [NATIVE / "src" / s for s in CORE_SOURCES] + [NATIVE / "tests" / "stress_main.cpp"]
    deps = srcs + _headers() + [Path(__file__)]
    if not force and _fresh(out, deps, [kind]):
        return out
    out.parent.mkdir(parents=True, exist_ok=True)
    opt = ["-O2"] if kind == "plain" else ["-O1", "-g", "-fno-omit-frame-pointer"]
    _run(["g++", "-std=c++17", *opt, *SANITIZERS[kind], f"-I{NATIVE / 'include'}", f"-I{ROCM / 'include'}",
          *[str(x) for x in srcs], "-o", str(out), "-ldl", "-lpthread", "-lssl", "-lcrypto"])
    return _done(out, deps, [kind])


def build_probe(force: bool = False) -> Path | None:
    hipcc = shutil.which("hipcc") or str(ROCM / "bin" / "hipcc")
    if not Path(hipcc).exists():
        return None
    out = PKG / f"_probe{EXT}"
    srcs = [NATIVE / "hip" / "probe.hip"]
    deps = srcs + _headers() + [Path(__file__)]
    if not force and _fresh(out, deps, [ARCH]):
        return out
    BUILD.mkdir(parents=True, exist_ok=True)
    _run([hipcc, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared",
          "-fvisibility=hidden", "-Wno-unused-result", f"-I{NATIVE / 'include'}", *_pybind_includes(),
          str(srcs[0]), "-o", str(out)])
    return _done(out, deps, [ARCH])


def build_all(force: bool = False, hip: bool = True) -> dict[str, str]:
    res = {"core": str(build_core(force)), "topo_cli": str(build_topo_cli(force))}
    if hip:
        p = build_probe(force)
        res["probe"] = str(p) if p else ""
    return res


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--no-hip", action="store_true")
    ap.add_argument("--sanitize", choices=["address", "thread", "undefined"])
    ap.add_argument("--stress", choices=list(SANITIZERS), help="build the native stress driver")
    a = ap.parse_args()
    if a.stress:
        print(build_stress(a.stress, force=a.force))
        return
    if a.sanitize:
        print(build_core(force=a.force, sanitize=a.sanitize))
        return
    for k, v in build_all(force=a.force, hip=not a.no_hip).items():
        print(f"{k}: {v}")


if __name__ == "__main__":
    main()
