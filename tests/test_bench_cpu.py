"""Host-side measurement logic (no GPU): algorithmic work per launch, the CPU-core count
the baseline uses, and bench.py's multi-rank launcher refusing a rank-count mismatch."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_conv_cost_matches_survey_table():
    from compressai import _ledger
    from compressai._native import ConvGeom

    # g_a[2] of bmshj2018-hyperprior q1 at B=16: Conv2d(128,128,k5,s2) 128x128 -> 64x64 = 53.7 GFLOP
    g = ConvGeom(16, 128, 128, 128, 128, 64, 64, 5, 2, 2, 0, 0)
    fl, nb = _ledger.conv_cost(g, 2, 0)
    assert abs(fl - 53.687e9) < 1e7
    assert nb == 2 * 16 * 128 * 128 * 128 + 2 * 16 * 64 * 64 * 128 + 2 * 128 * 128 * 25
    # the transposed twin (g_s deconv 128->128, 64x64 -> 128x128) does the same MACs
    gt = ConvGeom(16, 128, 64, 64, 128, 128, 128, 5, 2, 2, 1, 1)
    assert _ledger.conv_cost(gt, 2, 0)[0] == fl
    # weight gradient: fp32 read-modify-write of dW
    assert _ledger.conv_cost(g, 2, 2)[1] == nb - 2 * 128 * 128 * 25 + 8 * 128 * 128 * 25


def test_whole_step_flops_match_survey():
    """Sum of the conv + GDN FLOPs of the C2 training step recomputed from the layer table = SURVEY.md's
    33.93 GFLOP per patch (fwd 11.41)."""
    from compressai import _ledger
    from compressai._native import ConvGeom

    N, M, B = 128, 192, 1
    convs = [  # (cin, cout, H, k, s, transposed, needs dgrad)
        (3, N, 256, 5, 2, False, False), (N, N, 128, 5, 2, False, True), (N, N, 64, 5, 2, False, True),
        (N, M, 32, 5, 2, False, True),
        (M, N, 16, 3, 1, False, True), (N, N, 16, 5, 2, False, True), (N, N, 8, 5, 2, False, True),
        (N, N, 4, 5, 2, True, True), (N, N, 8, 5, 2, True, True), (N, M, 16, 3, 1, False, True),
        (M, N, 16, 5, 2, True, True), (N, N, 32, 5, 2, True, True), (N, N, 64, 5, 2, True, True),
        (N, 3, 128, 5, 2, True, True),
    ]
    fwd = train = 0.0
    for cin, cout, H, k, s, t, dg in convs:
        if t:
            OH = (H - 1) * s - 2 * (k // 2) + k + 1
        else:
            OH = (H + 2 * (k // 2) - k) // s + 1
        g = ConvGeom(B, cin, H, H, cout, OH, OH, k, s, k // 2, 1 if t else 0, int(t))
        f = _ledger.conv_cost(g, 2, 0)[0]
        fwd += f
        train += f * (3 if dg else 2)
    gdn_px = [128 * 128, 64 * 64, 32 * 32, 32 * 32, 64 * 64, 128 * 128]
    fwd += sum(2.0 * p * N * N for p in gdn_px)
    train += sum(2.0 * p * N * N * 3 for p in gdn_px)       # fwd + dx + dgamma contractions (norm reused)
    assert abs(fwd / 1e9 - 11.41) < 0.1, fwd / 1e9
    assert abs(train / 1e9 - 33.93) < 0.35, train / 1e9


def test_host_cores_is_positive_and_bounded():
    sys.path.insert(0, ROOT)
    import bench

    n = bench.host_cores()
    assert 1 <= n <= (os.cpu_count() or 1)


def test_bench_refuses_rank_mismatch():
    """--gpus 2 under an environment that already says WORLD_SIZE=1 must not report a 1-rank run as 2 GPUs."""
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1"],
                       env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode != 0
    assert "--gpus 2 but the job has 1 ranks" in (r.stdout + r.stderr)


def test_dominant_class_sums_launches_of_one_kernel():
    """bench.py's dominant_class: the kernel class with the largest SUMMED time wins over the single longest
    launch (cheng2020: hundreds of short convs vs one Adam launch), with its class-level roofline fraction."""
    sys.path.insert(0, ROOT)
    import bench

    class E:
        def __init__(self, kernel, ms, flops, nbytes, roof):
            self.kernel, self.ms, self.flops, self.nbytes, self._roof = kernel, ms, flops, nbytes, roof

        def roofline_ms(self):
            return self._roof

    class L:
        entries = [E("adam_fused_kernel", 0.05, 0, 1e8, 0.02)] + [E("conv_small_kernel", 0.02, 1e9, 1e6, 0.001)] * 10

    d = bench.dominant_class(L())
    assert d["kernel"] == "conv_small_kernel" and d["launches"] == 10
    assert abs(d["ms_per_step"] - 0.2) < 1e-9 and abs(d["frac"] - 0.05) < 1e-9
    assert abs(d["share_of_instrumented"] - 0.2 / 0.25) < 1e-4


def test_pmc_traffic_only_for_the_measured_build(tmp_path, monkeypatch):
    """bench.py's roofline `traffic` comes from a committed rocprofv3 record only when that record measured the
    libcai.so this process runs (lib_sha256); a record of another build gives traffic None and says so."""
    import json

    sys.path.insert(0, ROOT)
    import bench

    monkeypatch.setattr(bench, "lib_build", lambda: "aaaa")
    prof = tmp_path / "profiles"
    prof.mkdir()
    rec = {"workload": "w", "kernel": "k", "shape": "s", "hbm_bytes_per_launch": 123, "lib_sha256": "aaaa"}
    (prof / "pmc_traffic.json").write_text(json.dumps([rec]))
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    assert bench.pmc_traffic("w", "k", "s")[0] == 123
    monkeypatch.setattr(bench, "lib_build", lambda: "bbbb")
    t, note = bench.pmc_traffic("w", "k", "s")
    assert t is None and "another build" in note
    assert bench.pmc_traffic("w", "k2", "s")[0] is None
