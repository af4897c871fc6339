"""Doc-sharded CLIs end to end on the GPU: the index, quantize and rank
CLIs launched by torchrun with 2 ranks produce byte-identical files to one process.
The test box has one GPU, so both ranks share it and the retrieval exchange runs
over gloo host tensors (parallel.exchange_backend); on an 8-GPU node every rank owns
its GPU and the same code path all-gathers over RCCL.  The merge is di_topk_merge on
the GPU either way."""
import json
import os
import socket
import subprocess
import sys
import tempfile
from pathlib import Path

import pytest
import torch

import encoder_ref
from conftest import GOLDEN, ROOT

pytestmark = pytest.mark.gpu


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _torchrun(module, args, world=2, timeout=240, extra_env=None):
    """world > 0: torchrun with `world` ranks; 0: one plain process.  PYTHONHASHSEED is
    fixed: query terms are a set (process_query), whose iteration order -- the
    reference's first-touch tie order -- follows the hash seed."""
    env = dict(os.environ, PYTHONPATH=str(ROOT), OMP_NUM_THREADS="4", PYTHONHASHSEED="0",
               **(extra_env or {}))
    run = ([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
            f"--nproc-per-node={world}", "--master-addr", "127.0.0.1",
            f"--master-port={_port()}"] if world else [sys.executable])
    cmd = run + ["-m", f"improving_learned_index_amd.{module}"] + args
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, "\n".join(l for l in r.stderr.splitlines()
                                         if "[rank" in l or "Error" in l)[-8000:]


@pytest.fixture(scope="module")
def ckpt(tmp_path_factory):
    from improving_learned_index_amd import _lib

    if _lib.device_count() < 1:
        pytest.fail("no HIP device visible (GPU test run without a GPU)")
    fx = json.loads((GOLDEN / "encoder_xlmr_small.json").read_text())
    sd = encoder_ref.seeded_state_dict(fx["state_dict_shapes"], fx["seed"], fx["std"])
    path = tmp_path_factory.mktemp("ckpt") / "DeepImpact_latest.pt"
    torch.save({"model_state_dict": sd, "optimizer_state_dict": {}, "step": 0,
                "batch_size": 0}, path)
    return fx, path


def test_index_cli_two_ranks_equals_one(ckpt):
    from improving_learned_index_amd import index as index_cli

    fx, path = ckpt
    texts = [t for t in fx["texts"] if t] * 3  # 21 passages: shards of 10 and 11
    with tempfile.TemporaryDirectory() as td:
        td = Path(td)
        coll = td / "collection.tsv"
        coll.write_text("".join(f"{i}\t{t}\n" for i, t in enumerate(texts)))
        common = ["--collection_path", str(coll), "--model_checkpoint_path", str(path),
                  "--tokenizer_path", str(GOLDEN / "tokenizer.json"), "--max_length",
                  str(fx["max_length"]), "--precision", "fp32", "--process_batch_size", "4",
                  "--num_processes", "1"]
        index_cli.main(common + ["--output_file_path", str(td / "one.index")])
        _torchrun("index", common + ["--output_file_path", str(td / "two.index")])
        assert (td / "two.index").read_bytes() == (td / "one.index").read_bytes()
        assert not list(td.glob("*.part*"))
        # no launcher: the plain CLI fans out to child ranks itself (--gpus 2 on this
        # 1-GPU box; on an 8-GPU node the default is every visible GPU)
        _torchrun("index", common + ["--output_file_path", str(td / "self.index"), "--gpus",
                                     "2"], world=0)
        assert (td / "self.index").read_bytes() == (td / "one.index").read_bytes()
        assert not list(td.glob("*.part*"))


def test_quantize_cli_two_ranks_equals_one():
    from improving_learned_index_amd.quantize import quantize_file

    src = GOLDEN / "q254.index"
    with tempfile.TemporaryDirectory() as td:
        td = Path(td)
        quantize_file(src, td / "one")
        _torchrun("quantize", ["-i", str(src), "-o", str(td / "two")])
        assert (td / "two").read_bytes() == (td / "one").read_bytes() == \
            (GOLDEN / "q254.quantized").read_bytes()
        _torchrun("quantize", ["-i", str(src), "-o", str(td / "two7"), "-m", "7"], world=3)
        quantize_file(src, td / "one7", max_val=7.0)
        assert (td / "two7").read_bytes() == (td / "one7").read_bytes()


def _same_run(got: str, want: str):
    g, w = got.splitlines(), want.splitlines()
    for i, (a, b) in enumerate(zip(g, w)):
        assert a == b, (i, a, b, len(g), len(w))
    assert len(g) == len(w), (len(g), len(w))


def test_rank_cli_two_ranks_equals_one():
    from improving_learned_index_amd.inverted_index import InvertedIndexCreator

    fx = json.loads((GOLDEN / "score.json").read_text())
    with tempfile.TemporaryDirectory() as td:
        td = Path(td)
        InvertedIndexCreator(GOLDEN / "collection.quantized", td / "index").run()
        qf = td / "queries.tsv"
        texts = [" ".join(t.lstrip("▁") for t in q) for q in fx["queries"]]
        texts = [t for t in texts if t.strip()]  # (an empty query line does not parse)
        qf.write_text("".join(f"q{i}\t{t}\n" for i, t in enumerate(texts)))
        args = ["--index_path", str(td / "index"), "--queries_path", str(qf),
                "--tokenizer_path", str(GOLDEN / "tokenizer.json")]
        _torchrun("rank", args + ["--output_path", str(td / "one.tsv")], world=0)
        _torchrun("rank", args + ["--output_path", str(td / "two.tsv")])
        _same_run((td / "two.tsv").read_text(), (td / "one.tsv").read_text())
        _torchrun("rank", args + ["--output_path", str(td / "self.tsv"), "--gpus", "2"], world=0)
        _same_run((td / "self.tsv").read_text(), (td / "one.tsv").read_text())
        # the RCCL exchange itself (one rank owns the GPU: nccl), DI_FORCE_DIST=1
        _torchrun("rank", args + ["--output_path", str(td / "rccl.tsv")], world=1,
                  extra_env={"DI_FORCE_DIST": "1"})
        _same_run((td / "rccl.tsv").read_text(), (td / "one.tsv").read_text())
        # ... with the pruned two-round exchange forced at one rank: its device branch
        # (torch.topk over the samples, the pack / unpack scatters, the padded round-2
        # all_gather over nccl) -- the code every multi-GPU retrieve of configs[2]/[3] runs
        _torchrun("rank", args + ["--output_path", str(td / "rccl_pruned.tsv")], world=1,
                  extra_env={"DI_FORCE_DIST": "1", "DI_EXCHANGE": "pruned"})
        _same_run((td / "rccl_pruned.tsv").read_text(), (td / "one.tsv").read_text())
        _torchrun("rank", args + ["--output_path", str(td / "three.tsv"), "--top_k", "7"],
                  world=3)
        _torchrun("rank", args + ["--output_path", str(td / "one7.tsv"), "--top_k", "7"],
                  world=0)
        _same_run((td / "three.tsv").read_text(), (td / "one7.tsv").read_text())


def test_rank_cli_long_queries_two_ranks_equals_one():
    """Queries of 257..700 known terms through the sharded rank CLI (device pointers,
    wide keys, all-gather, GPU merge): the same run file as one process, which
    test_index_gpu pins to the oracle.  (The 256-term limit of round 2 made this path
    write garbage lines; now a rejected query raises instead, see test_index_gpu.)"""
    import numpy as np

    rng = np.random.default_rng(17)
    n_terms = 900
    with tempfile.TemporaryDirectory() as td:
        td = Path(td)
        lines = []
        for d in range(4000):
            ts = rng.choice(n_terms, size=int(rng.integers(0, 40)), replace=False)
            lines.append(", ".join(f"\u2581w{t}: {int(rng.integers(1, 256))}" for t in ts))
        (td / "coll.quantized").write_text("\n".join(lines) + "\n", encoding="utf-8")
        from improving_learned_index_amd.inverted_index import InvertedIndexCreator

        InvertedIndexCreator(td / "coll.quantized", td / "index").run()
        qs = [rng.choice(n_terms, size=int(rng.integers(257, 700)), replace=False)
              for _ in range(5)]
        qs += [rng.choice(n_terms, size=4, replace=False) for _ in range(5)]
        qf = td / "queries.tsv"
        qf.write_text("".join(f"q{i}\t{' '.join(f'w{t}' for t in q)}\n"
                              for i, q in enumerate(qs)))
        args = ["--index_path", str(td / "index"), "--queries_path", str(qf),
                "--tokenizer_path", str(GOLDEN / "tokenizer.json")]
        _torchrun("rank", args + ["--output_path", str(td / "one.tsv")], world=0)
        _torchrun("rank", args + ["--output_path", str(td / "two.tsv")])
        one = (td / "one.tsv").read_text()
        _same_run((td / "two.tsv").read_text(), one)
        per_q = {}
        for line in one.splitlines():
            qid, doc, rank_, score = line.split("\t")
            per_q.setdefault(qid, []).append((int(doc), int(score)))
        for i in range(5):  # the long queries hit far more than 1000 docs
            assert len(per_q[f"q{i}"]) == 1000
            sc = [s_ for _, s_ in per_q[f"q{i}"]]
            assert sc == sorted(sc, reverse=True) and sc[0] > 255


def test_bench_two_ranks_completes(tmp_path):
    """bench.py under torchrun with 2 ranks (sharing the test box's GPU over gloo) runs its
    rank-0-only text and rank_e2e legs beside the other rank's retrieve leg to one JSON line: the
    driver's N > 1 scaling runs take this path (a sharded quantizer inside rank 0's
    text legs once deadlocked it)."""
    env = dict(os.environ, PYTHONPATH=str(ROOT), OMP_NUM_THREADS="4")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", f"--master-port={_port()}", "bench.py", "--gpus", "2",
           "--legs", "retrieve,text,rank_e2e", "--steps", "1", "--warmup", "1", "--text-docs",
           "20000", "--queries", "512", "--no-cpu"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-4000:]
    line = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(line) == 1, r.stdout[-2000:]
    d = json.loads(line[0])
    assert d["n_gpus"] == 2 and d["unit"] == "queries/s" and d["value"] > 0
    assert d["quantize"]["docs"] == 20000 and d["index_create"]["value"] > 0
    # (rank 0 alone runs the rank CLI's path, unsharded, while rank 1 waits at the next leg)
    assert d["rank_e2e"]["run_file_lines"] == 512 * d["config"]["k"]
    assert d["ranks_seen"] == 2 and d["backend"] == "gloo"


def test_bench_gpus_flag_launches_ranks_itself():
    """Plain `python3 bench.py --gpus 2` (no launcher, as the driver may run it) starts
    its two ranks as a child torchrun and reports the ranks its all_gather saw; on this
    1-GPU box they share the GPU over gloo (an 8-GPU node takes RCCL)."""
    env = dict(os.environ, PYTHONPATH=str(ROOT), OMP_NUM_THREADS="4")
    env.pop("WORLD_SIZE", None)
    cmd = [sys.executable, "bench.py", "--gpus", "2", "--legs", "retrieve,text", "--steps", "1",
           "--warmup", "1", "--text-docs", "20000", "--queries", "512", "--no-cpu"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-4000:]
    line = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(line) == 1, r.stdout[-2000:]
    d = json.loads(line[0])
    assert d["n_gpus"] == 2 and d["ranks_seen"] == 2 and d["backend"] == "gloo"
    assert d["value"] > 0
    # the pruned exact exchange: each rank sends its first k / 2 keys + the extras above
    # the union's k-th (verdict r04: <= 0.6 k keys per query and rank)
    x = d["retrieve"]["exchange"]
    assert x["gathered_keys_per_query"] <= 0.6 * d["config"]["k"], x
    assert x["collective_ms_per_step"] > 0


def test_bench_single_rank_rccl_path():
    """The RCCL (nccl) branch of the multi-rank bench, rehearsed on the 1-GPU box: one
    torchrun rank with DI_FORCE_DIST=1 initialises the nccl process group and runs every
    collective of the N-rank path (barriers, the max-over-ranks time, the device
    all_gather of the per-shard top-k keys and the GPU merge of the gathered lists) --
    the path the 8-GPU scaling run takes, whose gloo rehearsals cover only host tensors."""
    env = dict(os.environ, PYTHONPATH=str(ROOT), OMP_NUM_THREADS="4", DI_FORCE_DIST="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
           "--master-addr", "127.0.0.1", f"--master-port={_port()}", "bench.py", "--gpus", "1",
           "--legs", "retrieve,retrieve_shard", "--steps", "2", "--warmup", "1",
           "--queries", "512", "--no-cpu"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-4000:]
    line = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(line) == 1, r.stdout[-2000:]
    d = json.loads(line[0])
    assert d["backend"] == "nccl" and d["ranks_seen"] == 1 and d["n_gpus"] == 1
    assert d["value"] > 0 and d["retrieve_shard"]["value"] > 0
    assert "the first 20 queries equal the oracle" in r.stderr
    assert d["retrieve"]["exchange"]["gathered_keys_per_query"] <= d["config"]["k"]


def test_visible_gpus_matches_the_runtime():
    """The CLIs' runtime-free GPU count (KFD topology + openable render nodes) agrees
    with the HIP runtime's on this box."""
    import torch

    from improving_learned_index_amd import parallel

    assert parallel.visible_gpus() == torch.cuda.device_count()


def test_bench_single_rank_rccl_pruned_exchange():
    """verdict r5 #1: the pruned exchange's device / RCCL branch on the GPU box.  One
    torchrun rank, DI_FORCE_DIST=1 (nccl process group) and DI_EXCHANGE=pruned: rounds
    1-2 run on device tensors over nccl every step; the merged lists of the last step
    must equal the scorer's own (one shard: the exchange + merge is the identity), and
    the plain path is timed beside it.  (At one rank every key of the only list is in
    the global top-k, so round 2 sends all k of them after the k / g samples; the key
    savings need >= 2 ranks: test_exchange_cpu, test_bench_gpus_flag_launches_ranks_itself.)"""
    env = dict(os.environ, PYTHONPATH=str(ROOT), OMP_NUM_THREADS="4", DI_FORCE_DIST="1",
               DI_EXCHANGE="pruned")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
           "--master-addr", "127.0.0.1", f"--master-port={_port()}", "bench.py", "--gpus", "1",
           "--legs", "retrieve,retrieve_shard", "--steps", "3", "--warmup", "1", "--no-cpu"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-4000:]
    line = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(line) == 1, r.stdout[-2000:]
    d = json.loads(line[0])
    assert d["backend"] == "nccl" and d["ranks_seen"] == 1
    k = d["config"]["k"]
    for leg in ("retrieve", "retrieve_shard"):
        x = d[leg]["exchange"]
        assert x["path"] == "pruned", x
        assert x["merged_equals_local_at_one_rank"] is True, x
        g = max(1, min(64, k // 4))
        assert x["gathered_keys_per_query"] <= k // g + k, x
        assert x["collective_ms_per_step"] > 0
        assert x["other_path"]["path"] == "plain" and x["other_path"]["collective_ms_per_step"] > 0
    print(json.dumps({leg: d[leg]["exchange"] for leg in ("retrieve", "retrieve_shard")}))
