"""spawn() for GPU tests whose ranks share the box's one GPU."""
from jax_distributed_tuts_amd.runtime.launch import spawn


def spawn8(fn, ws, *args):
    """spawn() of ``ws`` ranks on the box's one GPU.  Every failure fails the test --
    8-rank cases included: the in-kernel wait bounds grow with the ranks sharing the
    card (runtime/dist.spin_timeout_s), so a rank whose queue is scheduled late is waited
    for instead of being reported, and a timeout that still fires is a real failure."""
    spawn(fn, ws, *args, gpu=True)
