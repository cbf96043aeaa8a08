"""Build the in-tree native artefacts.

* `build_hip()`    — compiles every `csrc/*.hip` for gfx950 with hipcc into
                     `ops/lib/libkagent_hip.so` (one object per source, compiled in parallel,
                     then linked).  Cross-compiles without a GPU.
* `build_runtime()`— compiles the C++ host runtime (`runtime/*.cpp`: tokenizer trie, paged-KV
                     block manager, batch-metadata builder) into `runtime/_native*.so` via pybind11.

Both are incremental (rebuild only when a source is newer than the output).
"""
from __future__ import annotations

import concurrent.futures as cf
import glob
import os
import subprocess
import sys
import sysconfig

PKG = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(PKG, "csrc")
LIB_DIR = os.path.join(PKG, "ops", "lib")
HIP_LIB = os.path.join(LIB_DIR, "libkagent_hip.so")
RUNTIME_DIR = os.path.join(PKG, "runtime")
ARCH = os.environ.get("KA_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


def _newer(srcs, out) -> bool:
    if not os.path.exists(out):
        return True
    t = os.path.getmtime(out)
    return any(os.path.getmtime(s) > t for s in srcs)


def _run(cmd):
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError("command failed: %s\n%s" % (" ".join(cmd), r.stdout))
    return r.stdout


def file_flags(src: str):
    """Per-source hipcc flags from a `// KA_HIPCC_FLAGS: ...` line in the file's header comment."""
    with open(src) as f:
        for i, line in enumerate(f):
            if line.startswith("// KA_HIPCC_FLAGS:"):
                return line.split(":", 1)[1].split()
            if i > 40:
                break
    return []


def build_hip(force: bool = False, verbose: bool = False, extra_flags=(), out: str = "") -> str:
    """out: another library path (an A/B build with `extra_flags`, e.g. -DKA_GM_SCHED=0, loaded only by
    diagnostic runs: ops/_hip.py KA_HIP_LIB + KA_HIP_LIB_DIAG=1); its objects go next to it."""
    srcs = sorted(glob.glob(os.path.join(CSRC, "*.hip")))
    headers = glob.glob(os.path.join(CSRC, "*.h"))
    lib = out or HIP_LIB
    os.makedirs(os.path.dirname(lib), exist_ok=True)
    if not force and not _newer(srcs + headers, lib):
        return lib
    obj_dir = os.path.join(os.path.dirname(lib), "obj") if out else os.path.join(LIB_DIR, "obj")
    os.makedirs(obj_dir, exist_ok=True)
    flags = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-munsafe-fp-atomics",
             "-Wno-unused-result", *extra_flags]

    def compile_one(src):
        obj = os.path.join(obj_dir, os.path.basename(src) + ".o")
        if force or _newer([src] + headers, obj):
            _run([HIPCC, *flags, *file_flags(src), "-c", src, "-o", obj])
        return obj

    jobs = min(len(srcs), int(os.environ.get("MAX_JOBS", "8")))
    with cf.ThreadPoolExecutor(max(1, jobs)) as ex:
        objs = list(ex.map(compile_one, srcs))
    tmp = lib + ".tmp"
    _run([HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", *objs, "-o", tmp])
    if not out:
        check_lgkm_windows(verbose)
    os.replace(tmp, lib)
    if verbose:
        print("built", lib)
    return lib


# Kernels whose k-loops read LDS fragments with inline-asm ds_reads and wait for them with a COUNTED
# `s_waitcnt lgkmcnt(N)` (gemm_mfma.hip KA_GM_PIPE 2, gemm_big.hip): the count is only right if the
# compiler puts no LGKM operation of its own (scalar/kernarg load, LDS access, flat access, message)
# between those reads and the wait.  hipcc cannot see the asm, so a different compiler version or
# scheduling choice could silently break it; check_lgkm_windows() re-verifies every build.
LGKM_CHECKED = {"gemm_mfma.hip": r"gemm_kernel", "gemm_big.hip": r"gemm256_kernel"}


def lgkm_window_violations(asm_text: str, func_pat: str):
    """(number of asm fragment reads seen, [(function, line, instruction)] of compiler-issued LGKM
    operations inside an asm-read window: after an asm ds_read, before the next lgkmcnt wait)."""
    import re
    bad, fn, in_asm, pending, nreads = [], None, False, False, 0
    for ln, line in enumerate(asm_text.splitlines(), 1):
        m = re.match(r"^(_Z\S+):", line)
        if m:
            fn = m.group(1) if re.search(func_pat, m.group(1)) else None
            pending = False
            continue
        if fn is None:
            continue
        t = line.strip()
        if t.startswith(";;#ASMSTART"):
            in_asm = True
            continue
        if t.startswith(";;#ASMEND"):
            in_asm = False
            continue
        if not t or t.startswith(";") or t.startswith("."):
            continue
        op = t.split()[0]
        if in_asm and op.startswith("ds_read"):
            pending, nreads = True, nreads + 1
            continue
        if op == "s_waitcnt" and "lgkmcnt" in t:
            pending = False
            continue
        if pending and (op.startswith(("s_load", "s_buffer_load", "flat_", "s_sendmsg"))
                        or (op.startswith("ds_") and not in_asm)):
            bad.append((fn, ln, t))
    return nreads, bad


def mfma_span_valu(asm_text: str, func_pat: str):
    """[(function, line, instruction)] of compiler-issued VALU instructions between the first and the
    last inline-asm MFMA of each matching function.  gemm_big's k-loop is all asm (MFMAs with pinned
    AGPR accumulators, fragment reads, LDS-DMA): hipcc cannot see those MFMAs read their A / B VGPRs
    for several cycles after issue, so a VALU write it schedules there may overwrite an operand still
    being read (seen: a mask register reusing a dead A fragment's VGPR -> sparse wrong outputs)."""
    import re
    bad, fn, lines = [], None, []

    def flush():
        if fn is None:
            return
        idx = [i for i, (_, t, a) in enumerate(lines) if a and t.startswith("v_mfma")]
        if idx:
            for ln, t, a in lines[idx[0]:idx[-1]]:
                if not a and t.startswith("v_") and not t.startswith("v_mfma"):
                    bad.append((fn, ln, t))

    in_asm = False
    for ln, line in enumerate(asm_text.splitlines(), 1):
        m = re.match(r"^(_Z\S+):", line)
        if m:
            flush()
            fn, lines = (m.group(1) if re.search(func_pat, m.group(1)) else None), []
            continue
        t = line.strip()
        if t.startswith(";;#ASMSTART"):
            in_asm = True
        elif t.startswith(";;#ASMEND"):
            in_asm = False
        elif fn is not None and t and not t.startswith((";", ".")):
            lines.append((ln, t, in_asm))
    flush()
    return bad


def check_lgkm_windows(verbose: bool = False) -> None:
    """Compile the LGKM_CHECKED sources to device assembly and fail the build on any violation."""
    for name, pat in LGKM_CHECKED.items():
        src = os.path.join(CSRC, name)
        out = os.path.join(LIB_DIR, "obj", name + ".s")
        _run([HIPCC, "-O3", "-std=c++17", f"--offload-arch={ARCH}", "--cuda-device-only", "-S",
              *file_flags(src), src, "-o", out])
        with open(out) as f:
            nreads, bad = lgkm_window_violations(f.read(), pat)
        if nreads == 0:
            raise RuntimeError(f"{name}: no asm fragment reads found in the {pat} kernels (checker out of date?)")
        if bad:
            raise RuntimeError(f"{name}: compiler LGKM operations inside counted asm-read windows "
                               f"(the lgkmcnt counts would be wrong): {bad[:5]}")
        if name == "gemm_big.hip":
            with open(out) as f:
                valu = mfma_span_valu(f.read(), pat)
            if valu:
                raise RuntimeError(f"{name}: compiler VALU inside the asm-MFMA k-loop (operand WAR hazard "
                                   f"against in-flight MFMAs): {valu[:5]}")
        if verbose:
            print(f"lgkm windows ok: {name} ({nreads} asm reads)")


def build_runtime(force: bool = False, verbose: bool = False) -> str:
    srcs = sorted(glob.glob(os.path.join(RUNTIME_DIR, "*.cpp")))
    if not srcs:
        return ""
    import pybind11

    suffix = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
    out = os.path.join(RUNTIME_DIR, "_native" + suffix)
    if not force and not _newer(srcs + glob.glob(os.path.join(RUNTIME_DIR, "*.h")), out):
        return out
    inc = [pybind11.get_include(), sysconfig.get_paths()["include"]]
    cmd = ["g++", "-O3", "-std=c++17", "-shared", "-fPIC", "-fvisibility=hidden", *srcs,
           *[f"-I{i}" for i in inc], "-o", out + ".tmp"]
    if os.environ.get("KA_SANITIZE"):
        cmd[1:1] = ["-fsanitize=address,undefined", "-fno-omit-frame-pointer", "-g"]
    _run(cmd)
    os.replace(out + ".tmp", out)
    if verbose:
        print("built", out)
    return out


def build_all(force: bool = False, verbose: bool = True):
    return build_hip(force, verbose), build_runtime(force, verbose)


if __name__ == "__main__":
    build_all(force="--force" in sys.argv)
