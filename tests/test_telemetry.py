"""In-process telemetry on CPU: GPU-counter rates / exposition (exporter/pmc_sampler.py with a
fake counter source) and the per-rank metrics merge of multi-process pods
(exporter/rank_metrics.py)."""
import os

from aws_k8s_ansible_provisioner_amd.exporter import rank_metrics
from aws_k8s_ansible_provisioner_amd.exporter.pmc_sampler import PMCSampler

NAMES = ["GRBM_COUNT", "GRBM_GUI_ACTIVE", "SQ_BUSY_CYCLES", "SQ_VALU_MFMA_BUSY_CYCLES",
         "TCC_EA0_RDREQ_sum"]


def _fake(sampler, seq):
    it = iter(seq)
    sampler.names = list(NAMES)
    sampler._read = lambda: list(next(it))


def test_pmc_rates_cumulative_counters(monkeypatch):
    """Device-counting reads that accumulate: rates are deltas over the read interval; the
    first read's back-to-back probe classifies the semantics."""
    s = PMCSampler(interval_s=1.0, labels={"rank": "3"})
    s.settle_s = 0.0
    base = [2e9, 1e9, 5e8, 1e9, 1e8]
    _fake(s, [[0.0] * 5, base, base, [b * 2 for b in base]])  # start read, settle, probe
    t = iter([10.0, 10.0, 12.0])
    monkeypatch.setattr("time.monotonic", lambda: next(t))
    assert s.once() and s.cumulative is True and s.rates == {}
    assert s.once()
    assert abs(s.rates["GRBM_COUNT"] - 1e9) < 1  # (4e9 - 2e9) / 2 s
    d = s.derived()
    assert abs(d["gpu_busy_ratio"] - 0.5) < 1e-9
    # MFMA busy over every SIMD vs XCD-summed GUI_ACTIVE: 1e9 / (1e9 x 32 CUs/XCD x 4 SIMDs)
    assert abs(d["mfma_busy_ratio"] - 1.0 / 128) < 1e-9
    assert abs(d["mem_read_bytes_per_second"] - 0.5e8 * 128) < 1
    text = s.text()
    assert 'akap_gpu_pmc_up{rank="3"} 1' in text
    assert 'akap_gpu_pmc_rate{counter="GRBM_COUNT",rank="3"}' in text or \
        'akap_gpu_pmc_rate{rank="3",counter="GRBM_COUNT"}' in text
    assert "akap_gpu_pmc_gpu_busy_ratio" in text


def test_pmc_rates_per_read_counters(monkeypatch):
    """Reads that restart from zero: each read is the interval's own count."""
    s = PMCSampler(interval_s=1.0)
    s.settle_s = 0.0
    _fake(s, [[0.0] * 5, [2e9, 1e9, 5e8, 1e9, 1e8], [1e3, 1e3, 1e3, 1e3, 1e3],
              [4e9, 1e9, 5e8, 0, 2e8]])
    t = iter([10.0, 10.0, 14.0])
    monkeypatch.setattr("time.monotonic", lambda: next(t))
    assert s.once() and s.cumulative is False
    assert s.once()
    assert abs(s.rates["GRBM_COUNT"] - 1e9) < 1 and s.derived()["mfma_busy_ratio"] == 0.0


def test_pmc_failure_is_reported_not_raised():
    s = PMCSampler(lib="/nonexistent/libakap_pmc.so")
    assert s.once() is False and s.failures == 1
    assert "akap_gpu_pmc_up 0" in s.text()
    assert "not loadable" in s.status()


def test_rank_metrics_merge_and_labels(tmp_path, monkeypatch):
    """Follower ranks' telemetry files merged into rank 0's /metrics: one HELP/TYPE per family,
    every rank's samples together, rank labels added, stale files and rank 0 skipped."""
    monkeypatch.setattr(rank_metrics, "DIR", str(tmp_path))
    fam = ("# HELP akap_kernel_profiler_up up\n# TYPE akap_kernel_profiler_up gauge\n"
           "akap_kernel_profiler_up 1\n"
           "# TYPE akap_kernel_time_seconds_total counter\n"
           'akap_kernel_time_seconds_total{kernel="k"} 2.5\n')
    for r in (1, 2):
        w = rank_metrics.RankMetricsWriter("tp-29500", r,
                                           [lambda r=r: rank_metrics.add_labels(fam, {"rank": r})])
        w.write_once()
    rank_metrics.RankMetricsWriter("other-group", 1, [lambda: fam]).write_once()
    old = rank_metrics._path("tp-29500", 3)
    open(old, "w").write(fam)
    os.utime(old, (1, 1))  # stale: ignored
    peers = rank_metrics.read_peers("tp-29500")
    assert len(peers) == 2
    mine = rank_metrics.add_labels(fam, {"rank": 0})
    text = rank_metrics.merge([mine] + peers)
    lines = text.splitlines()
    assert lines.count("# TYPE akap_kernel_profiler_up gauge") == 1
    assert lines.count("# TYPE akap_kernel_time_seconds_total counter") == 1
    up = [i for i, ln in enumerate(lines) if ln.startswith("akap_kernel_profiler_up{")]
    assert len(up) == 3 and up == list(range(up[0], up[0] + 3))  # contiguous family
    assert 'akap_kernel_time_seconds_total{kernel="k",rank="2"} 2.5' in lines
    assert 'akap_kernel_profiler_up{rank="0"} 1' in lines
