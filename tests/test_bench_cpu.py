"""CPU tests of bench.py's contract plumbing: `--gpus N` outside torchrun starts N ranks itself
(world-2 gloo dry run: two ranks, one JSON line from rank 0 with n_gpus = 2), and the C2/C3/C4
positives come from the reference's own triples."""
import json
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def _json_lines(out):
    return [json.loads(l) for l in out.splitlines() if l.startswith("{")]


def test_gpus2_self_launches_two_ranks_one_line():
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dry-run", "--steps", "3"],
                       capture_output=True, text=True, timeout=180, env=env, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = _json_lines(p.stdout)
    assert len(lines) == 1, p.stdout
    line = lines[0]
    # the driver's contract keys, as the N > 1 line carries them
    assert {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
            "vs_baseline", "dtype", "data", "config"} <= set(line)
    assert line["metric"] == bench.METRIC and line["scaling"] == "weak" and line["higher_is_better"] is True
    assert {"workload", "parallelism"} <= set(line["config"]) and line["config"]["parallelism"] == "replicas2"
    assert line["n_gpus"] == 2 and line["steps"] == 3 and line["dry_run"]
    assert line["rank_sum"] == 1  # ranks 0 and 1 both joined the process group
    # the N > 1 row-sharded record: per-variant step times, the selected form, and every rank's diagnosis
    rs = line["yago3_10_rowshard"]
    assert set(rs["variants"]) == {"torchcomm_python", "one_stream_1chunk", "two_stream_2chunk"}
    assert rs["selected"] == bench.ROWSHARD_DEFAULT and rs["n_ranks_seen"] == 2
    assert [r["rank"] for r in rs["per_rank"]] == [0, 1]
    assert all(set(bench.ROWSHARD_RANK_KEYS) <= set(r) for r in rs["per_rank"])
    assert rs["native_status"] == "ok" and rs["native_matches_torchcomm"] is True


def test_rowshard_report_falls_back_to_the_python_path():
    """A native communicator that failed its check, or a native step whose outputs differ from the
    torch.distributed path's, leaves the Python path's numbers as the selected ones."""
    w = bench.WORKLOADS["c4s"]
    var = {"torchcomm_python": 2e-4, "one_stream_1chunk": 1e-4, "two_stream_2chunk": 1.2e-4}
    ok = bench.rowshard_report(w, 8, 20, var, [], 8, "ok", True)
    assert ok["selected"] == "one_stream_1chunk" and abs(ok["ms_per_step"] - 0.1) < 1e-9
    assert ok["triples_per_s"] == (512 * 1024 + 512) * 8 / 1e-4
    bad = bench.rowshard_report(w, 8, 20, var, [], 8, "ok", False)
    assert bad["selected"] == "torchcomm_python"
    err = bench.rowshard_report(w, 8, 20, {"torchcomm_python": 2e-4}, [], None, "native communicator: boom", None)
    assert err["selected"] == "torchcomm_python" and abs(err["ms_per_step"] - 0.2) < 1e-9


def test_gpus1_dry_run_is_single_process():
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--dry-run", "--steps", "2"],
                       capture_output=True, text=True, timeout=120, env=env, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-2000:]
    (line,) = _json_lines(p.stdout)
    assert line["n_gpus"] == 1


def test_c2_positives_are_wn18rr_train_triples():
    w = bench.WORKLOADS["c2"]
    pos, src = bench.positives(w, 0, 3)
    assert "wn18rr" in src
    tri = bench.load_triples(w)
    assert tri.shape == (86835, 3)
    assert all(p.shape == (512, 3) for p in pos)
    # every positive is a real training triple, in the RandomState(0) permutation order
    perm = np.random.RandomState(0).permutation(len(tri))
    assert np.array_equal(pos[0], tri[perm[:512]])
    assert np.array_equal(pos[2], tri[perm[1024:1536]])
    assert tri[:, 0].max() < w["nentity"] and tri[:, 1].max() < w["nrelation"]


def test_positives_split_over_ranks_are_disjoint():
    w = bench.WORKLOADS["c2"]
    a, _ = bench.positives(w, 0, 2, world=2)
    b, _ = bench.positives(w, 1, 2, world=2)
    tri = bench.load_triples(w)
    perm = np.random.RandomState(0).permutation(len(tri))
    assert np.array_equal(a[0], tri[perm[0:512]]) and np.array_equal(b[0], tri[perm[512:1024]])
    assert np.array_equal(a[1], tri[perm[1024:1536]])


def test_c3_c4_positives_from_reference_splits():
    for key, n in (("c3", 38001), ("c4", 10000)):
        w = bench.WORKLOADS[key]
        tri = bench.load_triples(w)
        assert tri.shape == (n, 3)
        assert tri[:, 0].max() < w["nentity"] and tri[:, 2].max() < w["nentity"]
        assert tri[:, 1].max() < w["nrelation"]


def test_pmc_traffic_is_tied_to_the_library_build(tmp_path, monkeypatch):
    """roofline.traffic comes from the committed PMC summary only while the loaded libkge_hip.so is built from
    the sources the passes ran (kge_source_hash, recorded by scripts/pmc_summary.py); any other build reports it
    stale."""
    prof = tmp_path / "profiles"
    prof.mkdir()
    rows = [{"kernel": "step_fwd_xcd_kernel<4, true, 4, 4>", "hbm_read_bytes_corrected": 800.0, "hbm_write_bytes": 2.0},
            {"kernel": "step_fwd_xcd_kernel<4, false, 4, 4>", "hbm_read_bytes_corrected": 900.0, "hbm_write_bytes": 2.0},
            {"kernel": "neg_rows_kernel", "hbm_read_bytes_corrected": 10.0, "hbm_write_bytes": 1.0}]
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    monkeypatch.setattr(bench, "loaded_source_hash", lambda: "abc")
    (prof / "pmc_c2.json").write_text(json.dumps({"source_hash": "abc", "kernels": rows}))
    t, src = bench.pmc_traffic("c2", ["step_fwd_xcd_kernel", "neg_rows_kernel"])
    assert t == (802.0 + 902.0) / 2 + 11.0 and src.endswith("pmc_c2.json")
    (prof / "pmc_c2.json").write_text(json.dumps({"source_hash": "other", "kernels": rows}))
    t, src = bench.pmc_traffic("c2", ["step_fwd_xcd_kernel"])
    assert t is None and src.startswith("stale")
    t, src = bench.pmc_traffic("c9", ["step_fwd_xcd_kernel"])
    assert t is None


def test_main_gives_ranks_disjoint_positives():
    """main() builds each rank's batches with its world size (make_inputs(..., world=world)), so at world 2
    the two ranks' first batches hold disjoint slices of the permuted WN18RR train triples."""
    import inspect
    src = inspect.getsource(bench.main)
    assert "make_inputs(w, rank, device, world=world)" in src
    w = bench.WORKLOADS["c2"]
    (a0, _), = bench.rank_batches(w, 0, 1, world=2)[0]
    (b0, _), = bench.rank_batches(w, 1, 1, world=2)[0]
    tri = bench.load_triples(w)
    perm = np.random.RandomState(0).permutation(len(tri))
    assert np.array_equal(a0, tri[perm[0:512]]) and np.array_equal(b0, tri[perm[512:1024]])
    ia = set(perm[0:512].tolist())
    assert not ia & set(perm[512:1024].tolist())


def test_cpu_baseline_runs_on_the_gpu_lines_inputs():
    """The CPU baseline's sample is the first rows of the timed batch 0 (rank 0): WN18RR train triples and
    the RandomState(2) negatives, not separate random ids."""
    w = bench.WORKLOADS["c2"]
    pos, neg, src = bench.cpu_baseline_inputs(w, 64)
    (p0, n0), = bench.rank_batches(w, 0, 1)[0]
    assert np.array_equal(pos.numpy(), p0[:64]) and np.array_equal(neg.numpy(), n0[:64])
    assert "wn18rr_ids.npz" in src
    assert np.array_equal(n0, np.random.RandomState(2).randint(w["nentity"], size=(512, 256)))


def test_sharded_watchdog_prints_the_headline_and_exits_nonzero():
    """A hung row-sharded side section (its first RCCL use at N > 1) must not cost the headline line: the
    watchdog prints rank 0's line, marked, and leaves with a non-zero status (the harness sees the hang). The
    line is serialised before the section runs: keys the section adds later are not in it."""
    import subprocess
    import sys
    code = ("import bench, time; line = {'metric': 'm', 'value': 1.0}; "
            "bench.sharded_watchdog(line, 0, 0.5); line['late'] = 1; time.sleep(30)")
    r = subprocess.run([sys.executable, "-c", code], cwd=ROOT, capture_output=True, text=True, timeout=60)
    assert r.returncode == bench.SHARDED_TIMEOUT_STATUS != 0
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["value"] == 1.0 and "timeout" in out["yago3_10_rowshard_error"] and "late" not in out
