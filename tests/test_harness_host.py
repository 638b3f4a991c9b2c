"""Host-side harness logic, no GPU: the BER sweep's resume keying and seeds
(modulations_amd/ber.py) and bench.py's fail-fast rank spawner."""
import argparse
import json
import os
import sys
import textwrap
import time

import pytest

from modulations_amd import ber

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _ns(**kw):
    d = dict(mod="256QAM", n=752, rate="1/3", algo="max-log", iterations=8, interleaver="reference",
             codewords=1000, seed=2025)
    d.update(kw)
    return argparse.Namespace(**d)


def test_resume_reuses_points_of_the_same_sweep(tmp_path):
    out = str(tmp_path / "sweep.json")
    cfg = ber.sweep_config(_ns())
    assert ber.load_resume(out, cfg) == {}
    recs = [{"ebn0_db": 2.0, "bit_errors": 5}, {"ebn0_db": -1.0, "bit_errors": 9}]
    ber.save_results(out, cfg, recs)
    got = ber.load_resume(out, ber.sweep_config(_ns()))
    assert sorted(got) == [-1.0, 2.0] and got[2.0]["bit_errors"] == 5


@pytest.mark.parametrize("change", [dict(mod="16QAM"), dict(n=212), dict(rate="1/2"), dict(algo="log-map"),
                                    dict(iterations=4), dict(interleaver="valid-perm"), dict(codewords=10),
                                    dict(seed=1)])
def test_resume_refuses_another_configuration(tmp_path, change):
    out = str(tmp_path / "sweep.json")
    ber.save_results(out, ber.sweep_config(_ns()), [{"ebn0_db": 0.0}])
    with pytest.raises(ValueError, match="another sweep configuration"):
        ber.load_resume(out, ber.sweep_config(_ns(**change)))


def test_resume_refuses_the_unkeyed_format(tmp_path):
    out = str(tmp_path / "old.json")
    json.dump([{"ebn0_db": 0.0, "bit_errors": 1}], open(out, "w"))
    with pytest.raises(ValueError, match="old format"):
        ber.load_resume(out, ber.sweep_config(_ns()))


def test_point_seed_depends_on_the_value_not_the_grid():
    assert ber.parse_points("-2:10:1")[4] == 2.0 and ber.parse_points("0:4:2")[1] == 2.0
    assert ber.ebn0_seed(2025, 2.0) == ber.ebn0_seed(2025, 2.0000)
    seeds = {ber.ebn0_seed(2025, e) for e in ber.parse_points("-2:10:0.5")}
    assert len(seeds) == 25                                         # distinct per point
    assert ber.ebn0_seed(2025, 1.0) != ber.ebn0_seed(2026, 1.0)
    assert all(0 <= s < 2 ** 64 for s in seeds)


def _rank_script(tmp_path, body):
    p = tmp_path / "rank.py"
    p.write_text(textwrap.dedent(body))
    return str(p)


def _bench():
    sys.path.insert(0, ROOT)
    import bench
    return bench


def test_spawn_ranks_kills_the_others_when_one_fails(tmp_path):
    script = _rank_script(tmp_path, """
        import os, sys, time
        if os.environ["RANK"] == "1":
            sys.exit(3)
        time.sleep(600)                  # rank 0 would wait at a barrier forever
    """)
    t0 = time.monotonic()
    rc = _bench().spawn_ranks(2, argv=[], deadline=60, script=script, poll=0.05)
    assert rc == 3 and time.monotonic() - t0 < 30


def test_spawn_ranks_deadline_kills_a_stuck_job(tmp_path):
    script = _rank_script(tmp_path, """
        import os, time
        if os.environ["RANK"] == "0":
            raise SystemExit(0)         # one rank finishes, the other hangs
        time.sleep(600)
    """)
    t0 = time.monotonic()
    rc = _bench().spawn_ranks(2, argv=[], deadline=2.0, script=script, poll=0.05)
    assert rc == 124 and time.monotonic() - t0 < 30


def test_spawn_ranks_success_and_environment(tmp_path):
    out = tmp_path / "ranks"
    out.mkdir()
    script = _rank_script(tmp_path, f"""
        import os
        open(os.path.join({str(out)!r}, os.environ["RANK"]), "w").write(
            " ".join(os.environ[k] for k in ("LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR")))
    """)
    assert _bench().spawn_ranks(3, argv=[], deadline=60, script=script, poll=0.05) == 0
    assert sorted(os.listdir(out)) == ["0", "1", "2"]
    assert (out / "2").read_text() == "2 3 127.0.0.1"


def test_bench_rejects_rccl_ranks_on_one_gpu():
    import subprocess
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--all-on-device0"],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and "gloo" in r.stderr
