"""Per-file sharding and the vocabulary broadcast on a world_size-2 gloo group (CPU)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from whisperx_amd.distributed import (_decode_dictionary, _encode_dictionary, align_corpus,
                                      broadcast_dictionary, gather_results, host_topology, lpt_plan, pin_rank,
                                      rank_cpus, rank_cpus_numa, shard_files)


def test_shard_files_lpt_balanced_and_complete():
    durs = [60, 1, 45, 30, 30, 12, 5, 59, 2, 33]
    for world in (1, 2, 4, 8):
        shards = shard_files(durs, world)
        flat = sorted(i for s in shards for i in s)
        assert flat == list(range(len(durs)))
        loads = [sum(durs[i] for i in s) for s in shards]
        assert max(loads) - min(loads) <= max(durs)
    assert shard_files(durs, 2) == shard_files(list(durs), 2)  # deterministic


def test_shard_files_config4_corpus():
    import numpy as np

    rng = np.random.default_rng(4)
    d = np.exp(rng.uniform(np.log(60), np.log(3600), 40))
    d = d / d.sum() * 36000.0  # 10 h
    shards = shard_files(d.tolist(), 8)
    loads = [d[s].sum() for s in shards]
    assert max(loads) / (36000.0 / 8) < 1.25


def test_dictionary_codec_roundtrip():
    d = {"<pad>": 0, "<s>": 1, "|": 4, "e": 5, "'": 27, "ü": 40, "日": 41}
    assert _decode_dictionary(_encode_dictionary(d)) == d


def test_rank_cpus_disjoint_and_covering():
    for cpus in ([0, 1, 2, 3, 4, 5, 6, 7], list(range(16)), [3, 9, 12], list(range(0, 256, 2))):
        for world in (1, 2, 3, 4, 8):
            parts = [rank_cpus(cpus, r, world) for r in range(world)]
            if world <= len(cpus):
                assert sorted(c for p in parts for c in p) == sorted(cpus)
                assert all(p for p in parts)
                assert max(map(len, parts)) - min(map(len, parts)) <= 1
            else:
                assert all(len(p) == 1 for p in parts)
    with pytest.raises(ValueError):
        rank_cpus([0, 1], 2, 2)


def test_rank_cpus_numa_split_and_fallback():
    topo = {"gpu_nodes": [0, 0, 0, 0, 1, 1, 1, 1], "node_cpus": {0: list(range(64)), 1: list(range(64, 128))}}
    aff = list(range(0, 128, 2))
    parts = [rank_cpus_numa(aff, r, 8, topo) for r in range(8)]
    assert sorted(c for p in parts for c in p) == aff  # disjoint, covering
    for r, p in enumerate(parts):
        assert p and set(p) <= set(topo["node_cpus"][topo["gpu_nodes"][r]])
    # the affinity misses node 1 entirely: every rank falls back to plain slices (no overlap)
    aff2 = list(range(16))
    assert [rank_cpus_numa(aff2, r, 8, topo) for r in range(8)] == [rank_cpus(aff2, r, 8) for r in range(8)]
    # unknown topology / fewer GPUs than ranks
    assert rank_cpus_numa(aff, 3, 8, None) == rank_cpus(aff, 3, 8)
    assert rank_cpus_numa(aff, 3, 8, {"gpu_nodes": [0, 1], "node_cpus": topo["node_cpus"]}) == rank_cpus(aff, 3, 8)


def _fake_sysfs(root, gpus, node_cpulists):
    """A KFD topology under `root`: one CPU agent, then GPUs [(pci bus, numa node)] in KFD order;
    node cpulists {node: "a-b,c"}."""
    base = root / "class/kfd/kfd/topology/nodes"
    (base / "0").mkdir(parents=True)
    (base / "0" / "properties").write_text("cpu_cores_count 64\nsimd_count 0\n")
    for i, (bus, node) in enumerate(gpus, start=1):
        (base / str(i)).mkdir()
        (base / str(i) / "properties").write_text(f"simd_count 1024\nlocation_id {bus << 8}\ndomain 0\n")
        dev = root / f"bus/pci/devices/0000:{bus:02x}:00.0"
        dev.mkdir(parents=True)
        (dev / "numa_node").write_text(f"{node}\n")
    for node, cl in node_cpulists.items():
        d = root / f"devices/system/node/node{node}"
        d.mkdir(parents=True)
        (d / "cpulist").write_text(cl + "\n")
    return str(root)


def test_host_topology_from_fake_sysfs(tmp_path, monkeypatch):
    """KFD nodes (CPU agents skipped), PCI location -> numa_node, node cpulists, visibility:
    ROCR_VISIBLE_DEVICES, then HIP_VISIBLE_DEVICES, or CUDA_VISIBLE_DEVICES only when HIP_ is
    unset; an unmappable entry (UUID, out of range) gives no topology rather than a wrong one."""
    for v in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        monkeypatch.delenv(v, raising=False)
    root = _fake_sysfs(tmp_path, [(0x0c, 1), (0x8c, 0), (0x1c, 1)], {0: "0-3,8-11", 1: "4-7,12-15"})
    topo = host_topology(root)
    assert topo["gpu_nodes"] == [1, 0, 1]
    assert topo["node_cpus"] == {0: [0, 1, 2, 3, 8, 9, 10, 11], 1: [4, 5, 6, 7, 12, 13, 14, 15]}
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "2,1")
    assert host_topology(root)["gpu_nodes"] == [1, 0]
    monkeypatch.setenv("CUDA_VISIBLE_DEVICES", "0")  # ignored while HIP_VISIBLE_DEVICES is set
    assert host_topology(root)["gpu_nodes"] == [1, 0]
    monkeypatch.delenv("HIP_VISIBLE_DEVICES")
    assert host_topology(root)["gpu_nodes"] == [1]
    monkeypatch.setenv("ROCR_VISIBLE_DEVICES", "1,2")  # applied first: CUDA's 0 -> KFD GPU 1
    assert host_topology(root)["gpu_nodes"] == [0]
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "GPU-5f1c2a3b")  # UUID: no reliable map
    assert host_topology(root) is None
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "7")  # out of range
    assert host_topology(root) is None
    assert host_topology(root, visible_only=False)["gpu_nodes"] == [1, 0, 1]
    assert host_topology(str(tmp_path / "missing")) is None


def test_pin_rank_node_model_with_fewer_visible_gpus(tmp_path, monkeypatch):
    """One visible GPU modelling rank r of an 8-GPU node: the KFD's full GPU list stands in
    (numa_source "node_model"), and the reason is recorded when nothing can be modelled."""
    for v in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        monkeypatch.delenv(v, raising=False)
    aff = sorted(os.sched_getaffinity(0))
    if len(aff) < 2:
        pytest.skip("needs two CPUs")
    half = len(aff) // 2
    cl = {0: ",".join(map(str, aff[:half])), 1: ",".join(map(str, aff[half:]))}
    root = _fake_sysfs(tmp_path / "n8", [(0x10 + 0x10 * i, i // 4) for i in range(8)], cl)
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "5")
    old = os.sched_getaffinity(0)
    try:
        for r in (0, 5):
            pin = pin_rank(r, 8, sysfs=root)
            os.sched_setaffinity(0, old)
            assert pin["numa_source"] == "node_model" and pin["numa"] == r // 4, pin
            assert set(pin["cpus"]) <= set(aff[:half] if r < 4 else aff[half:])
        pin = pin_rank(0, 8, sysfs=str(tmp_path / "missing"))
        os.sched_setaffinity(0, old)
        assert pin["numa"] is None and pin["numa_source"] is None and "KFD" in pin["numa_reason"], pin
        root2 = _fake_sysfs(tmp_path / "n2", [(0x10, 0), (0x20, 1)], cl)
        pin = pin_rank(0, 8, sysfs=root2)
        os.sched_setaffinity(0, old)
        assert pin["numa"] is None and "2 GPU(s)" in pin["numa_reason"], pin
    finally:
        os.sched_setaffinity(0, old)


def test_lpt_plan_config4():
    from whisperx_amd import synthetic

    plan = lpt_plan(synthetic.corpus_durations(4))
    assert set(plan) == {"1", "2", "4", "8"}
    assert plan["1"]["max_over_mean"] == 1.0
    for w in ("2", "4", "8"):
        assert 1.0 <= plan[w]["max_over_mean"] < 1.25


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _fake_numa(world):
    """The parent's CPUs as two NUMA nodes, GPUs crossed over them (GPU r on node 1 - r % 2)."""
    cpus = sorted(os.sched_getaffinity(0))
    half = len(cpus) // 2
    return {"gpu_nodes": [1 - r % 2 for r in range(world)], "node_cpus": {0: cpus[:half], 1: cpus[half:]}}


def _worker(rank, world, port, q, numa=False, sysfs=None):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    # before anything else, as bench.py's ranks do
    if sysfs:  # fewer visible GPUs than ranks: the node model
        os.environ["HIP_VISIBLE_DEVICES"] = "0"
        pin = pin_rank(rank, world, sysfs=sysfs)
    else:
        pin = pin_rank(rank, world, topology=_fake_numa(world) if numa else "auto")
    pin["affinity"] = sorted(os.sched_getaffinity(0))
    pin["torch_threads"] = torch.get_num_threads()
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        vocab = {"<pad>": 0, "|": 4, "e": 5, "t": 6, "ä": 33} if rank == 0 else None
        got = broadcast_dictionary(vocab, device=None)
        durs = [30.0, 10.0, 25.0, 5.0, 60.0]
        res = align_corpus([f"f{i}" for i in range(5)], lambda f: {"file": f, "rank": rank}, durs)
        q.put((rank, got, res, pin))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("numa", [False, True, "node_model"], ids=["host", "fake_numa", "fewer_visible_gpus"])
def test_gloo_world2_broadcast_and_gather(numa, tmp_path):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    sysfs = None
    if numa == "node_model":  # a 2-GPU node whose ranks each see one GPU: GPU r on node 1 - r
        cpus = sorted(os.sched_getaffinity(0))
        half = len(cpus) // 2
        sysfs = _fake_sysfs(tmp_path, [(0x10, 1), (0x20, 0)],
                            {0: ",".join(map(str, cpus[:half])), 1: ",".join(map(str, cpus[half:]))})
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q, numa is True, sysfs)) for r in range(2)]
    for p in procs:
        p.start()
    outs = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    outs.sort(key=lambda x: x[0])
    for rank, got, res, pin in outs:
        assert got == {"<pad>": 0, "|": 4, "e": 5, "t": 6, "ä": 33}
    # per-rank host pinning: disjoint CPU sets covering the parent's affinity, pools sized to them
    parent = sorted(os.sched_getaffinity(0))
    sets = [o[3]["affinity"] for o in outs]
    if len(parent) >= 2:
        assert not set(sets[0]) & set(sets[1])
        assert sorted(sets[0] + sets[1]) == parent
    for o in outs:
        assert o[3]["affinity"] == o[3]["cpus"]
        assert 1 <= o[3]["torch_threads"] <= len(o[3]["cpus"])
    if numa and len(parent) >= 2:  # each rank on its GPU's (fake) node: rank 0 -> node 1
        topo = _fake_numa(2)
        for r, o in enumerate(outs):
            assert set(o[3]["cpus"]) <= set(topo["node_cpus"][topo["gpu_nodes"][r]])
            assert o[3]["numa"] == topo["gpu_nodes"][r]
            assert o[3]["numa_source"] == ("node_model" if numa == "node_model" else "given")
    merged = outs[0][2]
    assert outs[1][2] is None
    assert sorted(merged) == [0, 1, 2, 3, 4]
    shards = shard_files([30.0, 10.0, 25.0, 5.0, 60.0], 2)
    for r in (0, 1):
        for i in shards[r]:
            assert merged[i] == {"file": f"f{i}", "rank": r}


@pytest.mark.gpu
def test_rccl_world1_device_broadcast_and_allreduce():
    """The RCCL branch on the GPU: a world-size-1 "nccl" (= RCCL) group, the dictionary's
    device-tensor broadcast (forced past the world-of-one shortcut) and bench._allreduce on
    device tensors (max and sum) — the collectives the 8-GPU bench runs, on one GPU."""
    import bench

    assert torch.cuda.is_available()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0, world_size=1,
                            device_id=dev)
    try:
        assert dist.get_backend() == "nccl"
        vocab = {"<pad>": 0, "|": 4, "e": 5, "ß": 37, "日": 41}
        assert broadcast_dictionary(vocab, device=dev, force=True) == vocab
        old = bench._allreduce.dev
        bench._allreduce.dev = dev
        try:
            assert bench._allreduce([1.5, -2.0], "max") == [1.5, -2.0]
            assert bench._allreduce([3.0, 4.0], "sum") == [3.0, 4.0]
        finally:
            bench._allreduce.dev = old
        dist.barrier()
    finally:
        dist.destroy_process_group()
