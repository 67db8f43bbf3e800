"""Host sanitizer sweep of the planner and the issue scheduler
(tools/plan_bounds.cpp): schedule.cpp / issue.cpp / trees.cpp built with g++
-fsanitize=address,undefined, every algorithm (reduce family, allgather, bcast,
gather / scatter / alltoall) x P x rank (x root) x
sizes (ragged reduce-scatter blocks) x in / out of place x transport settings
(flat allgather, flat reduce-scatter, multi-tree, relay, chunked), every
primitive of the plan and of the issue schedule checked to stay inside the
buffer it names (the caller's SBUF / RBUF under each collective's MPI
conventions, TMP0-2 within the plan's workspace, STAGE within the schedule's).
An out-of-range primitive would be an out-of-bounds access on the GPU."""
import os
import shutil
import subprocess
from concurrent.futures import ThreadPoolExecutor

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "pico_amd", "csrc")
EXE = os.path.join(ROOT, "tools", "_build", "plan_bounds")

ALGOS = [0, 1, 2, 3, 4, 5, 6, 7, 16, 17, 18, 19, 20, 21, 22, 23, 24, 32, 33,
         48, 49, 50, 51, 52, 53, 54, 55, 56, 57, 58, 59, 64, 65, 66, 67, 68, 69, 70, 80, 81, 82]
# the flat reduce-scatter / multi-tree algorithms also up to P = 16 (16-leaf trees)
P16 = [4, 5, 6, 20, 21, 22, 33]


@pytest.fixture(scope="module")
def exe():
    if shutil.which("g++") is None:
        pytest.skip("g++ not available")
    srcs = [os.path.join(CSRC, f) for f in ("schedule.cpp", "issue.cpp", "trees.cpp")]
    srcs.append(os.path.join(ROOT, "tools", "plan_bounds.cpp"))
    if not os.path.exists(EXE) or os.path.getmtime(EXE) < max(os.path.getmtime(s) for s in srcs + [
            os.path.join(CSRC, "bine_internal.h"), os.path.join(ROOT, "include", "bine_amd.h")]):
        os.makedirs(os.path.dirname(EXE), exist_ok=True)
        subprocess.run(["g++", "-O2", "-g", "-std=c++17", "-fsanitize=address,undefined",
                        "-fno-sanitize-recover=undefined", "-ffp-contract=off",
                        "-I" + os.path.join(ROOT, "include"), "-I" + CSRC, *srcs, "-o", EXE], check=True)
    return EXE


def test_plans_and_schedules_stay_in_bounds(exe):
    jobs = [(8, a) for a in ALGOS] + [(16, a) for a in P16]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1")

    def run(job):
        maxp, algo = job
        r = subprocess.run([exe, str(maxp), str(algo)], capture_output=True, text=True, timeout=600, env=env)
        return job, r

    with ThreadPoolExecutor(max_workers=min(6, os.cpu_count() or 1)) as ex:
        results = list(ex.map(run, jobs))
    for (maxp, algo), r in results:
        assert r.returncode == 0, f"algo {algo} P<={maxp}:\n{r.stdout[-500:]}\n{r.stderr[-3000:]}"
        assert "0 out of range" in r.stdout, r.stdout
