"""GPU tests for the HIP validation kernels (libnetop_hip.so, gfx950) and the RCCL path.

Numerics are checked against plain PyTorch fp32 references of the same op.
"""

import pytest

pytestmark = pytest.mark.gpu


def _ref_pattern(n, seed, rank):
    """fp32 reference of the device pattern (mirrors group_hash() / base_mult() / step_mult() /
    group_sum() in netop_hip.hip), written independently of collectives.pattern_reference."""
    import torch

    return _ref_at(torch.arange(n, dtype=torch.int64), seed, rank)


def _ref_at(i, seed, rank):
    """The same at the element indices ``i`` (an int64 tensor; any size of index)."""
    M32 = 0xFFFFFFFF
    g = i >> 3  # one hash per 8-element group
    h = ((g & M32) * 0x9E3779B1) & M32 ^ ((((g >> 32) & M32) * 0x85EBCA77) & M32)
    h ^= h >> 15
    h = (h * 0x2C1B3C6D) & M32
    h ^= h >> 12
    k = ((seed + 0x632BE5AB) & M32) * 0xC2B2AE3D & M32
    k2 = ((seed ^ 0x27D4EB2F) & M32) * 0x165667B1 & M32
    mult = (((k ^ (k >> 16)) | 1) + rank * ((((k2 ^ (k2 >> 15)) << 1) | 2) & M32)) & M32  # m_0 + rank d
    word = (h * mult) & M32  # rank's word; element i = field at bit 5 + 3 (i % 8)
    return (((word >> (5 + 3 * (i % 8))) & 7) - 4).float()


def test_fill_pattern_matches_reference(cuda_device):
    import torch

    from network_operator_amd.ops import hip

    n = 1 << 16
    t = torch.empty(n, dtype=torch.bfloat16, device=cuda_device)
    for rank in (0, 3):
        hip.fill_pattern(t, 77, rank)
        torch.testing.assert_close(t.float().cpu(), _ref_pattern(n, 77, rank), rtol=0, atol=0)


def test_expected_sum_and_verify(cuda_device):
    import torch

    from network_operator_amd.ops import hip

    n = (1 << 20) + 8
    for world in (8, 20):  # 20: three 9-rank slot flushes in the SWAR sum
        ref = sum(_ref_pattern(n, 5, r) for r in range(world))
        t = torch.empty(n, dtype=torch.bfloat16, device=cuda_device)
        hip.fill_expected_sum(t, 5, world)
        torch.testing.assert_close(t.float().cpu(), ref, rtol=0, atol=0)
        assert hip.verify_sum(t, 5, world) == 0
        t[12345] += 1
        t[-1] += 1
        assert hip.verify_sum(t, 5, world) == 2


def test_pattern_kernels_cover_every_element_across_workgroup_chunks(cuda_device):
    """The fill / verify walk gives each workgroup one contiguous chunk (a multiple of 256
    vectors) of a buffer larger than one chunk per workgroup: every element is written once with
    the right value, and a wrong element on either side of a chunk edge, or the very last one,
    is counted."""
    import torch

    from network_operator_amd.ops import hip

    nv = 3 * 4096 * 256 + 37  # vectors: more than 16 workgroups per CU x 256 lanes can take at once
    n = nv * 8
    t = torch.full((n,), float("nan"), dtype=torch.bfloat16, device=cuda_device)
    hip.fill_expected_sum(t, 11, 3)
    ref = sum(_ref_pattern(n, 11, r) for r in range(3))
    torch.testing.assert_close(t.float().cpu(), ref, rtol=0, atol=0)
    assert hip.verify_sum(t, 11, 3) == 0
    cus = torch.cuda.get_device_properties(cuda_device).multi_processor_count
    per = -(-(-(-nv // min(cus * 16, -(-nv // 256)))) // 256) * 256  # vectors per workgroup chunk
    flips = sorted({8 * per - 1, 8 * per, 16 * per - 1, 16 * per, n - 1})
    for i in flips:
        t[i] += 1
    assert hip.verify_sum(t, 11, 3) == len(flips)


def test_pattern_kernels_index_past_32_bits(cuda_device):
    """64-bit indexing, sized for 288 GB of HBM: element offsets past 2^35 (group ids past 2^32,
    where the hash takes the high word) against the reference, and -- when the GPU has the room --
    one buffer of more than 2^32 16-byte vectors (64 GiB + 80 B) filled and verified whole, a
    flipped element at its very end counted."""
    import torch

    from network_operator_amd.ops import hip

    off = (1 << 35) + 4096
    t = torch.empty(1 << 12, dtype=torch.bfloat16, device=cuda_device)
    hip.fill_pattern_at(t, 21, 0, 3, elem_offset=off)
    idx = torch.arange(1 << 12, dtype=torch.int64) + off
    torch.testing.assert_close(t.float().cpu(), sum(_ref_at(idx, 21, r) for r in range(3)), rtol=0, atol=0)
    assert hip.verify_pattern_at(t, 21, 0, 3, off) == 0

    n = ((1 << 32) + 5) * 8
    free, _ = torch.cuda.mem_get_info(cuda_device)
    if free < 2 * n + (8 << 30):
        pytest.skip(f"{free >> 30} GiB free: the > 2^32-vector buffer needs {(2 * n) >> 30} GiB")
    big = torch.empty(n, dtype=torch.bfloat16, device=cuda_device)
    try:
        hip.fill_pattern(big, 3, 1)
        assert hip.verify_pattern_at(big, 3, 1, 1, 0) == 0
        probe = torch.tensor([0, (1 << 32) * 8 - 1, (1 << 32) * 8, n - 1], dtype=torch.int64)
        torch.testing.assert_close(big[probe.to(cuda_device)].float().cpu(), _ref_at(probe, 3, 1), rtol=0, atol=0)
        big[n - 1] += 1
        assert hip.verify_pattern_at(big, 3, 1, 1, 0) == 1
    finally:
        del big
        torch.cuda.empty_cache()


def test_copy_matches_torch(cuda_device):
    import torch

    from network_operator_amd.ops import hip

    src = torch.randn(3 << 20, dtype=torch.float32, device=cuda_device)
    dst = torch.empty_like(src)
    hip.copy(src, dst)
    torch.cuda.synchronize()
    assert torch.equal(src, dst)


def test_bad_buffers_rejected(cuda_device):
    import torch

    from network_operator_amd.ops import hip

    with pytest.raises(ValueError):
        hip.fill_pattern(torch.empty(7, dtype=torch.bfloat16, device=cuda_device), 1, 0)
    with pytest.raises(ValueError):
        hip.fill_pattern(torch.empty(8, dtype=torch.float32, device=cuda_device), 1, 0)


def test_xgmi_probe_loopback(cuda_device):
    from network_operator_amd.ops import hip

    r = hip.xgmi_probe(64 << 20, iters=3)
    assert r["gpus"] >= 1
    assert r["errors"] == 0
    assert r["aggregate_GBps"][0] > 100  # HBM loopback on one GPU is far above any link


def test_rccl_all_reduce_verified(cuda_device, single_rank_pg):
    from network_operator_amd.parallel import collectives as C

    ok, errors = C.verify_all_reduce(1 << 22, cuda_device)
    assert ok and errors == 0
    res = C.run_sweep("all_reduce", [1 << 20], iters=5, warmup=2, device=cuda_device)
    assert res[0].busbw_GBps == 0.0  # n = 1
    assert res[0].time_s > 0


def test_amd_smi_xgmi_links_visible(cuda_device):
    """The MI355X in an 8-GPU hive reports 7 xGMI links up (one slot is the disabled self-link)."""
    from network_operator_amd.ops import smi

    snap = smi.snapshot()
    assert snap["gpus"], snap
    g = snap["gpus"][0]
    assert len(g["xgmi_read_kb"]) == 8
    if "link_status" in g:
        assert g["link_status"].count("U") in (0, 7), g["link_status"]
    t = smi.traffic(snap, smi.snapshot())
    assert t["gpus"] and t["links_with_traffic"] == 0  # idle: nothing moved


def test_pattern_at_offsets(cuda_device):
    import torch

    from network_operator_amd.ops import hip

    n = 4096
    t = torch.empty(n, dtype=torch.bfloat16, device=cuda_device)
    hip.fill_pattern_at(t, 9, 2, 3, elem_offset=1024)
    ref = sum(_ref_pattern(n + 1024, 9, r)[1024:] for r in (2, 3, 4))
    torch.testing.assert_close(t.float().cpu(), ref, rtol=0, atol=0)
    assert hip.verify_pattern_at(t, 9, 2, 3, 1024) == 0
    assert hip.verify_pattern_at(t, 9, 2, 3, 1032) > 0


@pytest.mark.parametrize("op", ["all_reduce", "all_gather", "reduce_scatter", "broadcast", "alltoall"])
@pytest.mark.parametrize("inplace,graph", [(False, False), (True, False), (False, True)])
def test_native_rccl_bench(cuda_device, op, inplace, graph):
    from network_operator_amd.parallel import rccl_bench

    rows = rccl_bench.run(op=op, gpus=1, min_bytes=1024, max_bytes=4 << 20, factor=16, iters=5, warmup=1,
                          inplace=inplace, graph=graph, timeout=120)
    assert [r.bytes for r in rows] == [1024, 16384, 262144, 4194304]
    assert all(r.checked and r.wrong == 0 and r.time_us > 0 for r in rows)
    assert all(r.busbw_GBps == 0.0 for r in rows) or op == "broadcast"  # n=1 bus factor


def test_rccl_env_probe_runs_every_variant(cuda_device):
    """bench.py's --rccl-autotune / validate.py --tune-rccl path: every knob variant starts RCCL
    in a fresh process and completes; at n = 1 busbw is 0, so the defaults stay chosen."""
    from network_operator_amd.parallel import rccl_bench

    probes = rccl_bench.env_probe(1, 16 << 20, iters=3, timeout=60, budget_s=90)
    assert [p["env"] for p in probes] == list(rccl_bench.ENV_PROBES)
    assert all("busbw_GBps" in p and p["time_us"] > 0 for p in probes), probes
    assert rccl_bench.choose_env(probes)["chosen"] == {}


@pytest.mark.parametrize("ranks", [1, 3, 8])
def test_xgmi_allreduce_algorithm_virtual_ranks(cuda_device, ranks):
    """The n-rank two-shot algorithm (pull and push) with every rank mapped onto the one GPU:
    chunking, phase ordering and buffer reuse are checked exactly over three seeds per size."""
    from network_operator_amd.parallel import xgmi_allreduce as X

    rows = X.run(ranks=ranks, min_bytes=1000, max_bytes=32 << 20, factor=32, iters=2, warmup=1, timeout=180)
    assert {r["mode"] for r in rows} == {"pull", "push"}
    assert len(rows) == 2 * 4  # 1000 B .. 32 MB, x32
    for r in rows:
        assert r["ranks"] == ranks and r["wrong"] == 0, r
        assert r["bytes"] % (16 * ranks) == 0


def test_xgmi_probe_isolated_matches_the_in_process_fields(cuda_device):
    """bench.py runs the probe out of process (rank 0 must outlive a faulting probe)."""
    from network_operator_amd.ops import hip

    r = hip.xgmi_probe_isolated(32 << 20, iters=3, max_gpus=1, timeout=120)
    assert r["gpus"] == 1 and r["errors"] == 0 and r["push_errors"] == 0
    assert r["aggregate_GBps"][0] > 100 and r["push_aggregate_GBps"][0] > 100
    assert len(r["link_GBps"]) == 1


def test_xgmi_probe_push_loopback(cuda_device):
    from network_operator_amd.ops import hip

    r = hip.xgmi_probe_push(32 << 20, iters=3)
    assert r["gpus"] >= 1 and r["errors"] == 0
    assert r["push_aggregate_GBps"][0] > 100


@pytest.mark.parametrize("nsrc", [1, 2, 3, 8])
def test_sum_bf16_matches_torch_fp32(cuda_device, nsrc):
    """n-way bf16 sum (fp32 accumulation, RNE) against a PyTorch fp32 reference of the same op."""
    import torch

    from network_operator_amd.ops import hip

    g = torch.Generator(device="cpu").manual_seed(nsrc)
    n = (1 << 20) + 64
    srcs_cpu = [torch.randn(n, generator=g).to(torch.bfloat16) for _ in range(nsrc)]
    srcs = [s.to(cuda_device) for s in srcs_cpu]
    out = torch.empty(n, dtype=torch.bfloat16, device=cuda_device)
    hip.sum_bf16(srcs, out)
    torch.cuda.synchronize()
    acc = torch.zeros(n, dtype=torch.float32)
    for s in srcs_cpu:  # same order as the kernel: exact match expected
        acc += s.float()
    torch.testing.assert_close(out.cpu(), acc.to(torch.bfloat16), rtol=0, atol=0)
    # and within bf16 rounding of an order-independent fp64 reference
    ref = torch.stack([s.double() for s in srcs_cpu]).sum(0)
    torch.testing.assert_close(out.cpu().double(), ref, rtol=2 ** -7, atol=1e-6)


def test_sum_bf16_rejects_bad_args(cuda_device):
    import torch

    from network_operator_amd.ops import hip

    a = torch.zeros(16, dtype=torch.bfloat16, device=cuda_device)
    with pytest.raises(ValueError):
        hip.sum_bf16([a] * 9, a)
    with pytest.raises(ValueError):
        hip.sum_bf16([a, torch.zeros(24, dtype=torch.bfloat16, device=cuda_device)], a)


def test_fabric_validation_single_gpu(cuda_device, tmp_path):
    """validate.run on the 1-GPU box: topology from the real KFD and PCIe tree (the agent's
    NCCL_TOPO_FILE for this box must agree with it), probe, RCCL sweep, counters."""
    from network_operator_amd import validate
    from network_operator_amd.parallel import fabric_artifacts as FA

    art = tmp_path / "art"
    doc = FA.generate(str(art))  # the agent itself (discover --dry-run): rccl-topo.xml + rccl.env
    assert "error" not in doc, doc
    rep = validate.run(gpus=1, min_busbw=0, min_link_GBps=0, max_bytes=64 << 20, nfd_dir=str(tmp_path),
                       artifact_dir=str(art))
    assert rep["ok"], rep
    names = [c["check"] for c in rep["checks"] if c["check"] not in ("xgmi_link_state", "rail_pcie_links")]
    assert names[:6] == ["xgmi_topology", "gpu_nic_affinity", "rccl_topology_file", "xgmi_probe", "rccl_all_reduce",
                         "rccl_xgmi_links"]
    by = {c["check"]: c for c in rep["checks"]}
    # every GPU's links in gpu_metrics (the node's 8, though the job sees one): none down
    assert by["xgmi_link_state"]["ok"] and by["xgmi_link_state"]["links_up"] >= 7, by["xgmi_link_state"]
    # every rail's NIC and GPU PCIe link at what it supports (both box families: 32 GT/s x16)
    assert by["rail_pcie_links"]["ok"] and len(by["rail_pcie_links"]["links"]) == 8, by["rail_pcie_links"]
    assert by["rccl_all_reduce"]["artifacts_applied"] and by["rccl_all_reduce"]["rccl_env"]["NCCL_TOPO_FILE"]
    assert by["rccl_xgmi_links"]["rccl_dump"]["gpus"] == 1 and by["rccl_xgmi_links"]["rccl_dump"]["gpu_ancestry_equal"]
    assert names[-1] == "xgmi_direct_all_reduce"
    assert (tmp_path / validate.LABEL_FILE).read_text().startswith(validate.LABEL + "=true\n")


def test_fabric_validation_direct_check_without_pytorch(cuda_device, monkeypatch):
    """Check 5 as the validation image runs it (no PyTorch): the native harness, exact."""
    from network_operator_amd import validate

    monkeypatch.setattr(validate, "_have_torch", lambda: False)
    c = validate.direct_all_reduce_check(1, 64 << 20, 120)
    assert c["ok"] and c["wrong"] == 0 and "no PyTorch" in c["runner"], c
    assert [s["bytes"] for s in c["sizes"] if s["algo"] == "pull"][-1] <= 64 << 20


@pytest.mark.parametrize("pairs,nbytes,wg", [(1, 16, 0), (3, 4096 + 16, 0), (7, 3 << 20, 0), (8, (5 << 20) + 48, 1)])
def test_multi_copy_matches_torch(cuda_device, pairs, nbytes, wg):
    """One launch copying up to 8 pairs: sizes that need one, several and many workgroups per
    pair (the grid-stride indexing covers every vector exactly once), vs torch's copy."""
    import torch

    from network_operator_amd.ops import hip

    g = torch.Generator(device=cuda_device).manual_seed(pairs)
    srcs = [torch.randint(0, 256, (nbytes,), dtype=torch.uint8, device=cuda_device, generator=g) for _ in range(pairs)]
    dsts = [torch.zeros(nbytes, dtype=torch.uint8, device=cuda_device) for _ in range(pairs)]
    hip.multi_copy(srcs, dsts, wg_per_cu=wg)
    torch.cuda.synchronize()
    for s, d in zip(srcs, dsts):
        assert torch.equal(s, d)
    with pytest.raises(ValueError):
        hip.multi_copy(srcs[:1], [torch.zeros(nbytes + 16, dtype=torch.uint8, device=cuda_device)])
