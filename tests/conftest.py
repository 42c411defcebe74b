import os
import sys

# Import torch before any engine library so one HIP runtime (torch's) serves
# both torch device buffers and libopenr_spf_hip in the test process.
import torch  # noqa: F401,E402

# A LinkState degrades to its host path on a device error;
# in the test suite it must not: a GPU test that passed on the host path
# would not be evidence for the engine. test_gpu_degrade.py turns it back on
# for the LinkStates it tests.
os.environ["ODL_STRICT_ENGINE"] = "1"

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device)")
    config.addinivalue_line("markers", "slow: long-running (large topologies)")


# tests/test_gpu_multirank.py: the 2-rank bench rehearsal is started here,
# after collection and before any test touches the GPU in this process
# (ranks are never forked from a process that has initialised HIP).
MULTIRANK = {}


def _launch_ranks(topology):
    import socket
    import subprocess
    import tempfile
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    out = tempfile.NamedTemporaryFile("w+", suffix=".jsonl", delete=False)
    err = tempfile.NamedTemporaryFile("w+", suffix=".log", delete=False)
    env = dict(os.environ, OPENR_BENCH_BACKEND="gloo", OPENR_BENCH_SHARE_DEVICE="1",
               HSA_ENABLE_IPC_MODE_LEGACY="0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(port),
           os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1",
           "--topology", topology, "--roots", "0", "--dist-parity", "96", "--iso-reps", "1"]
    return dict(proc=subprocess.Popen(cmd, stdout=out, stderr=err, cwd=ROOT, env=env),
                out=out.name, err=err.name)


def pytest_collection_finish(session):
    if not any("test_gpu_multirank" in it.nodeid for it in session.items):
        return
    # unit-metric derive mode and weighted derive mode, two ranks each
    MULTIRANK.update(unit=_launch_ranks("fabric10k"), weighted=_launch_ranks("fabric10k-w"))
