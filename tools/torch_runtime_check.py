"""The engine under PyTorch's bundled HIP runtime: at N > 1 bench.py imports torch.distributed before
it loads the engine, and torch's libamdhip64.so.7 (and librccl) then serve the engine too (same
soname). Runs the smoke check and a short single-GPU bench line in that setting (one process)."""
import runpy
import sys

import torch  # noqa: F401  (loads torch's HIP runtime first)
import torch.distributed  # noqa: F401

sys.path.insert(0, ".")
import __graft_entry__ as g  # noqa: E402

g.smoke()
print("smoke under torch's HIP runtime: ok", flush=True)
sys.argv = ["bench.py", "--steps", "200", "--warmup", "20", "--no-cpu-baseline", "--fetch-rounds", "2",
            "--concurrent-rounds", "0", "--host-steps", "0", "--tier-rounds", "0"]
runpy.run_path("bench.py", run_name="__main__")
