"""Process-level guards that run without a GPU: bench.py's rank-count contract
(--gpus N against a launcher's WORLD_SIZE) and the HIP-runtime load-order guard of
_lib.lib() (torch's bundled libamdhip64 must be the one mapped)."""
import os
import subprocess
import sys

from conftest import ROOT


def _run(code_or_args, env=None, timeout=120):
    e = dict(os.environ, PYTHONPATH=str(ROOT))
    e.update(env or {})
    return subprocess.run([sys.executable] + code_or_args, cwd=ROOT, env=e,
                          capture_output=True, text=True, timeout=timeout)


def test_bench_refuses_world_size_gpus_mismatch():
    """A launcher's WORLD_SIZE that differs from --gpus exits non-zero before any GPU
    call (the driver would otherwise record n_gpus it did not ask for)."""
    r = _run(["bench.py", "--gpus", "4", "--legs", "retrieve"],
             env={"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0
    assert "WORLD_SIZE=2 but --gpus 4" in r.stderr
    r = _run(["bench.py", "--gpus", "0"])
    assert r.returncode != 0 and "--gpus must be >= 1" in r.stderr


def test_bench_self_launch_builds_the_torchrun_command(monkeypatch):
    """--gpus N without WORLD_SIZE starts a child torchrun of N ranks (never exec) and
    forwards exactly one JSON line; the child here is a stub that prints one."""
    sys.path.insert(0, str(ROOT))
    import importlib

    bench = importlib.import_module("bench")
    seen = {}

    class FakePopen:
        def __init__(self, cmd, **kw):
            seen["cmd"] = cmd
            self.stdout = iter(['log line\n', '{"n_gpus": 3}\n'])

        def wait(self):
            return 0

    import subprocess as sp

    monkeypatch.setattr(sp, "Popen", FakePopen)
    rc = bench.launch_ranks(3, ["--gpus", "3", "--steps", "2"])
    assert rc == 0
    cmd = seen["cmd"]
    assert cmd[1:3] == ["-m", "torch.distributed.run"]
    assert "--nproc-per-node=3" in cmd and "127.0.0.1" in cmd
    assert cmd[-4:] == ["--gpus", "3", "--steps", "2"]
    assert cmd[-5].endswith("bench.py")


def test_hip_runtime_guard_refuses_a_foreign_runtime_loaded_first():
    """An embedder that maps /opt/rocm's libamdhip64 before torch gets a clear error
    from _lib.lib() instead of a torch bound to the wrong runtime."""
    code = ("import ctypes, glob\n"
            "rt = sorted(glob.glob('/opt/rocm/lib/libamdhip64.so.*'))\n"
            "assert rt, 'no /opt/rocm HIP runtime'\n"
            "ctypes.CDLL(rt[0])\n"
            "from improving_learned_index_amd import _lib\n"
            "try:\n"
            "    _lib.lib()\n"
            "except RuntimeError as e:\n"
            "    print('GUARD', e)\n")
    r = _run(["-c", code])
    assert r.returncode == 0, r.stderr[-2000:]
    assert "GUARD a HIP runtime other than torch's is already loaded" in r.stdout


def test_hip_runtime_guard_maps_torchs_runtime_first():
    """Loading the library in a fresh process imports torch first, so exactly one HIP
    runtime -- torch's -- is mapped afterwards."""
    code = ("import sys\n"
            "from improving_learned_index_amd import _lib\n"
            "assert 'torch' not in sys.modules\n"
            "_lib.lib()\n"
            "import torch, os\n"
            "rts = _lib.hip_runtimes_mapped()\n"
            "tdir = os.path.realpath(os.path.join(os.path.dirname(torch.__file__), 'lib'))\n"
            "assert len(rts) == 1 and next(iter(rts)).startswith(tdir), rts\n"
            "print('OK')\n")
    r = _run(["-c", code])
    assert r.returncode == 0, r.stderr[-2000:]
    assert "OK" in r.stdout


def test_visible_gpus_counts_kfd_nodes_without_hip(tmp_path, monkeypatch):
    """The CLIs' fan-out count comes from the KFD topology and the render nodes this
    process can open (no HIP call), restricted by the *_VISIBLE_DEVICES lists."""
    from improving_learned_index_amd import parallel

    topo, dri = tmp_path / "nodes", tmp_path / "dri"
    dri.mkdir()
    for i, (simds, minor) in enumerate([(0, None), (304, 128), (304, 129), (304, 130)]):
        d = topo / str(i)
        d.mkdir(parents=True)
        props = f"cpu_cores_count 8\nsimd_count {simds}\n"
        if minor is not None:
            props += f"drm_render_minor {minor}\n"
        (d / "properties").write_text(props)
    for minor in (128, 129):  # renderD130 is not exposed to this "container"
        (dri / f"renderD{minor}").write_text("")
    assert parallel._kfd_gpu_nodes(topo, dri) == 2
    assert parallel._kfd_gpu_nodes(tmp_path / "absent", dri) is None
    monkeypatch.setattr(parallel, "_kfd_gpu_nodes", lambda: 2)
    monkeypatch.delenv("HIP_VISIBLE_DEVICES", raising=False)
    monkeypatch.delenv("CUDA_VISIBLE_DEVICES", raising=False)
    monkeypatch.delenv("ROCR_VISIBLE_DEVICES", raising=False)
    assert parallel.visible_gpus() == 2
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "1")
    assert parallel.visible_gpus() == 1
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "")
    assert parallel.visible_gpus() == 0
