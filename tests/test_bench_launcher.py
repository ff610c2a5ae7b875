"""CPU: bench.py's multi-rank path end to end -- the self-launch of N ranks
(torch.distributed.run on 127.0.0.1), gloo barriers, max-over-ranks timing and
the rank-0 JSON line -- with --rehearse's numpy stand-in for the GPU step."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env_extra=None):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, cwd=ROOT,
                          env=env, capture_output=True, text=True, timeout=300)


def _line(p):
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert p.returncode == 0, p.stderr[-2000:]
    assert len(lines) == 1, p.stdout
    return json.loads(lines[0])


def test_self_launch_two_ranks_strong_c4():
    j = _line(_run(["--gpus", "2", "--rehearse", "--steps", "3", "--warmup", "1"]))
    assert j["n_gpus"] == 2 and j["rehearsal"] is True
    assert j["scaling"] == "strong"
    assert j["global_groups"] == 1 << 20 and j["groups_covered"] == 1 << 20
    assert j["value"] > 0


def test_self_launch_weak():
    j = _line(_run(["--gpus", "2", "--rehearse", "--scaling", "weak", "--groups", "1000",
                    "--steps", "2", "--warmup", "0"]))
    assert j["n_gpus"] == 2 and j["groups_covered"] == 2000 and j["scaling"] == "weak"


def test_single_rank_defaults_weak():
    j = _line(_run(["--rehearse", "--steps", "2", "--warmup", "0"]))
    assert j["n_gpus"] == 1 and j["scaling"] == "weak" and j["groups_covered"] == 65536


def test_world_size_mismatch_is_an_error():
    p = _run(["--gpus", "8", "--rehearse"], {"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert p.returncode != 0 and "WORLD_SIZE=1" in p.stderr
    assert not [l for l in p.stdout.splitlines() if l.startswith("{")]


def test_roofline_traffic_only_from_current_sources(tmp_path, monkeypatch):
    """roofline.traffic comes from a counter pass only while the kernel's
    sources still hash to the digest stamped into it; otherwise it is null and
    marked stale."""
    sys.path.insert(0, ROOT)
    import bench
    for which, kern in (("encode", "k_bs2_20_30"), ("decode", "k_decode_fused")):
        tj = {"kernel": kern, "groups": 65536, "hbm_bytes_per_launch": 123.0,
              "source_sha256": bench.kernel_source_sha(which)}
        p = tmp_path / f"{which}.json"
        p.write_text(json.dumps(tj))
        monkeypatch.setitem(bench.TRAFFIC, which, str(p))
        assert bench.roofline(which, kern + ": x", 1e9, 0.5, 65536)["traffic"] == 123.0
        p.write_text(json.dumps(dict(tj, source_sha256="0" * 64)))
        r = bench.roofline(which, kern + ": x", 1e9, 0.5, 65536)
        assert r["traffic"] is None and r["traffic_source"].startswith("stale")
