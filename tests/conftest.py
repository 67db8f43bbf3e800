import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)

# The GPU tests' own process shares the box's one GPU with the multi-process
# checks it starts; each HIP process holds up to GPU_MAX_HW_QUEUES queues per
# stream priority (+1), and past the GPU's hardware queue slots the scheduler
# time-slices them -- a rank whose queue is off the GPU stalls peers spinning
# for it (profiles/r4_queue_oversubscription.txt).  The box
# exports GPU_MAX_HW_QUEUES=4; this process takes 2 (read at HIP's first
# call, which comes later), the rank processes tests/_sub.py's share.
# BINE_TEST_QUEUES overrides.
os.environ["GPU_MAX_HW_QUEUES"] = os.environ.get("BINE_TEST_QUEUES", "2")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box)")
    config.addinivalue_line("markers", "slow: long CPU test")
