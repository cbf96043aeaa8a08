"""Which step of a bench rank's startup opens the GPU device (/dev/kfd)?  Prints, after each step,
whether this process (and its parent, e.g. torchrun) holds /dev/kfd."""
import os
import sys


def holds(pid=None):
    pid = os.getpid() if pid is None else pid
    found = False
    for fd in os.listdir(f"/proc/{pid}/fd"):
        try:
            found |= os.readlink(f"/proc/{pid}/fd/{fd}") == "/dev/kfd"
        except OSError:
            pass
    return found


def report(step):
    print(f"{step:40s} self={holds()} parent={holds(os.getppid())}", flush=True)


report("start")
import torch  # noqa: E402
report("import torch")
import torch.distributed as dist  # noqa: E402
report("import torch.distributed")
if "WORLD_SIZE" in os.environ:
    dist.init_process_group("gloo")
    report("init_process_group(gloo)")
    t = torch.zeros(1)
    dist.all_reduce(t)
    report("all_reduce(cpu tensor)")
    dist.monitored_barrier()
    report("monitored_barrier")
    dist.barrier()
    report("barrier")
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ai_agent_kubectl_amd.parallel import dp  # noqa: E402,F401
report("import parallel.dp")
n = torch.cuda.device_count()
report(f"torch.cuda.device_count() = {n}")
torch.cuda.is_available()
report("torch.cuda.is_available()")
