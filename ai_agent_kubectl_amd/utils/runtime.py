"""Process-level tuning for a serving process.

* GC: the engine keeps ~10^6 long-lived Python objects (the 128k-entry tokenizer trie, prompt
  caches); every full collection walks them.  `gc.freeze()` moves everything alive at start-up to
  the permanent generation and higher thresholds make young collections rarer under request load
  (measured on the ASGI path: 0.475 -> 0.27 ms per request).
* GIL: see engine.LLMEngine.start (switch interval).
"""
from __future__ import annotations

import gc
import os

_done = False


def tune_gc() -> None:
    global _done
    if _done or os.environ.get("KA_NO_GC_TUNING"):
        return
    gc.collect()
    gc.freeze()
    gc.set_threshold(100_000, 50, 100)
    _done = True


def _parse_cpulist(text: str) -> list:
    cpus = []
    for part in text.strip().split(","):
        if not part:
            continue
        lo, _, hi = part.partition("-")
        cpus.extend(range(int(lo), int(hi or lo) + 1))
    return cpus


def device_local_cpus(device_index: int) -> list:
    """CPUs on the NUMA node of GPU `device_index` (sysfs `local_cpulist` of its PCI function),
    intersected with this process's allowed set; [] when unknown."""
    import torch
    p = torch.cuda.get_device_properties(device_index)
    bdf = f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}.0"
    try:
        with open(f"/sys/bus/pci/devices/{bdf}/local_cpulist") as f:
            local = set(_parse_cpulist(f.read()))
    except (OSError, ValueError):
        return []
    return sorted(local & os.sched_getaffinity(0))


def pin_to_device_numa(device_index: int) -> list:
    """Pin this process to the CPUs next to its GPU (KA_NUMA_PIN=0 disables).

    On an 8-GPU node each DP replica's engine process launches kernels, copies step inputs and
    reads back sampled tokens every few ms; keeping it (and its API process) on the socket that
    hosts the GPU avoids cross-socket hops on every launch and readback.  Returns the CPU list
    (empty when nothing was changed)."""
    if os.environ.get("KA_NUMA_PIN", "1") != "1":
        return []
    try:
        cpus = device_local_cpus(device_index)
        if cpus and len(cpus) < len(os.sched_getaffinity(0)):
            pin_process(cpus)
            return cpus
    except Exception:  # pragma: no cover - best effort (no sysfs / restricted cpuset)
        pass
    return []


def pin_process(cpus) -> None:
    """sched_setaffinity for every thread of this process (pid 0 would pin only the caller;
    threads started later inherit the caller's mask)."""
    if not cpus:
        return
    for tid in os.listdir("/proc/self/task"):
        try:
            os.sched_setaffinity(int(tid), cpus)
        except OSError:  # pragma: no cover - thread exited meanwhile
            pass


def set_proc_name(name: str) -> None:
    """Name this process (/proc/<pid>/comm, at most 15 bytes: `ps`, `top`, psutil.name()) so the
    serving topology is readable from outside: ka-api-<i>, ka-replica-<i>, ka-tp-<i>.<r>."""
    try:
        import ctypes
        libc = ctypes.CDLL(None, use_errno=True)
        libc.prctl(15, ctypes.c_char_p(name.encode()[:15]), 0, 0, 0)   # PR_SET_NAME
    except (OSError, AttributeError):
        pass
