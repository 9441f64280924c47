"""Per-file data parallelism across the GPUs of a node.

One process per GPU (torchrun; LOCAL_RANK -> device).  Alignment/VAD work has no
cross-segment dependence, so files are partitioned across ranks and every rank aligns
its own files with no collective on the data path.  The only collectives:

  * broadcast_dictionary: the alignment model's character vocabulary from rank 0
    (a few hundred bytes; backend "nccl" = RCCL over xGMI on ROCm, "gloo" on CPU);
  * gather_results (optional): per-file result dicts to rank 0 (gather_object).

pin_rank splits the host CPUs between the ranks of a node (host CPU per rank —
Python orchestration and the aggregation — is the scaling limiter): each local rank gets a
disjoint slice of the process's CPU affinity, taken from its GPU's NUMA node when the host
exposes the KFD topology, and an intra-op thread pool of its share of the thread budget, so 8
ranks do not each start a pool over every core.

shard_files balances mixed-length corpora (BASELINE config 4: 40 files of 1-60 min)
longest-processing-time first: files sorted by duration (descending, index as tie
break), each assigned to the currently least-loaded rank (lowest rank on ties).
"""
from __future__ import annotations

import os
from typing import Dict, List, Optional, Sequence

import torch
import torch.distributed as dist


def shard_files(durations: Sequence[float], world_size: int) -> List[List[int]]:
    """LPT assignment of file indices to ranks; deterministic on every rank."""
    if world_size < 1:
        raise ValueError("world_size must be >= 1")
    order = sorted(range(len(durations)), key=lambda i: (-float(durations[i]), i))
    load = [0.0] * world_size
    shards: List[List[int]] = [[] for _ in range(world_size)]
    for i in order:
        r = min(range(world_size), key=lambda k: (load[k], k))
        shards[r].append(i)
        load[r] += float(durations[i])
    for s in shards:
        s.sort()
    return shards


def thread_budget() -> int:
    """Host threads this process may use: its CPU affinity, capped by OMP_NUM_THREADS (a
    shared box's os.cpu_count() counts the whole machine)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    omp = os.environ.get("OMP_NUM_THREADS", "")
    if omp.isdigit() and int(omp) > 0:
        n = min(n, int(omp))
    return max(n, 1)


def rank_cpus(cpus: Sequence[int], local_rank: int, local_world: int) -> List[int]:
    """Local rank's share of `cpus`: contiguous slices of the sorted list, disjoint across the
    ranks and together covering it (more ranks than CPUs: one CPU each, round robin)."""
    if local_world < 1 or not 0 <= local_rank < local_world:
        raise ValueError(f"local rank {local_rank} outside a node of {local_world}")
    cpus = sorted(int(c) for c in cpus)
    n = len(cpus)
    if n == 0:
        return []
    if local_world > n:
        return [cpus[local_rank % n]]
    return cpus[local_rank * n // local_world:(local_rank + 1) * n // local_world]


def _parse_cpulist(text: str) -> List[int]:
    out: List[int] = []
    for part in text.strip().split(","):
        if not part:
            continue
        lo, _, hi = part.partition("-")
        out.extend(range(int(lo), int(hi or lo) + 1))
    return out


def _visible(ids: List[int]) -> Optional[List[int]]:
    """The GPUs this process sees, as ROCr and HIP select them: ROCR_VISIBLE_DEVICES first, then
    HIP_VISIBLE_DEVICES, or CUDA_VISIBLE_DEVICES only when HIP_VISIBLE_DEVICES is unset (HIP
    honours one of the two, it does not compose them).  None when an entry cannot be mapped to
    a KFD GPU (a UUID, an out-of-range index): the caller then has no reliable GPU -> node map."""
    for names in (("ROCR_VISIBLE_DEVICES",), ("HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES")):
        v = next((os.environ[n] for n in names if os.environ.get(n, "").strip()), None)
        if v is None:
            continue
        try:
            ids = [ids[int(x)] for x in v.split(",") if x.strip() != ""]
        except (ValueError, IndexError):
            return None
    return ids


def host_topology(sysfs: str = "/sys", visible_only: bool = True) -> Optional[dict]:
    """{"gpu_nodes": NUMA node of each visible GPU in HIP's order, "node_cpus": {node: [cpus]}}
    from the KFD topology (GPU agents in node order, as ROCr enumerates them; PCI location ->
    the device's numa_node) filtered by ROCR_/HIP_/CUDA_VISIBLE_DEVICES (_visible), or None when
    the host does not expose it or the visibility list cannot be mapped.  visible_only=False
    keeps every GPU the KFD lists: the node's layout even when this process sees fewer GPUs
    (the host-share leg models rank 0 of an 8-GPU node on one visible GPU).  Reads sysfs only:
    no HIP call, so it can run before pinning."""
    base = os.path.join(sysfs, "class/kfd/kfd/topology/nodes")
    try:
        nodes = sorted(int(n) for n in os.listdir(base) if n.isdigit())
    except OSError:
        return None
    gpus: List[int] = []
    for n in nodes:
        try:
            with open(os.path.join(base, str(n), "properties")) as f:
                props = dict(line.split()[:2] for line in f if len(line.split()) >= 2)
        except OSError:
            continue
        if int(props.get("simd_count", "0")) <= 0:
            continue  # a CPU agent
        loc, dom = int(props.get("location_id", "0")), int(props.get("domain", "0"))
        bdf = f"{dom:04x}:{(loc >> 8) & 0xff:02x}:{(loc >> 3) & 0x1f:02x}.{loc & 7}"
        try:
            with open(os.path.join(sysfs, "bus/pci/devices", bdf, "numa_node")) as f:
                gpus.append(int(f.read().strip()))
        except (OSError, ValueError):
            gpus.append(-1)
    if visible_only:
        gpus = _visible(gpus)
    if not gpus or any(g < 0 for g in gpus):
        return None
    node_cpus = {}
    for g in set(gpus):
        try:
            with open(os.path.join(sysfs, f"devices/system/node/node{g}/cpulist")) as f:
                node_cpus[g] = _parse_cpulist(f.read())
        except OSError:
            return None
    return {"gpu_nodes": gpus, "node_cpus": node_cpus}


def rank_cpus_numa(cpus: Sequence[int], local_rank: int, local_world: int, topo: Optional[dict]) -> List[int]:
    """Local rank's CPUs from its GPU's NUMA node: the node's CPUs within `cpus`, split between
    the ranks whose GPUs share that node (rank_cpus).  Disjoint across ranks.  Falls back to
    rank_cpus over all of `cpus` for every rank when the topology is unknown, covers fewer GPUs
    than ranks, or any rank's node has none of `cpus` (a mixed rule could overlap)."""
    if local_world < 1 or not 0 <= local_rank < local_world:
        raise ValueError(f"local rank {local_rank} outside a node of {local_world}")
    allowed = set(int(c) for c in cpus)
    if topo and len(topo.get("gpu_nodes", [])) >= local_world:
        nodes = [topo["gpu_nodes"][r] for r in range(local_world)]
        share = {n: sorted(allowed & set(topo["node_cpus"].get(n, []))) for n in set(nodes)}
        if all(share[n] for n in nodes):
            peers = [r for r in range(local_world) if nodes[r] == nodes[local_rank]]
            return rank_cpus(share[nodes[local_rank]], peers.index(local_rank), len(peers))
    return rank_cpus(cpus, local_rank, local_world)


def pin_rank(local_rank: Optional[int] = None, local_world: Optional[int] = None,
             topology: Optional[dict] = "auto", sysfs: str = "/sys") -> dict:
    """Pin this rank to its disjoint CPU slice — on its GPU's NUMA node when the host exposes
    the topology (host_topology; `topology` overrides it, None disables it) — and size torch's
    intra-op pool to its share of the thread budget.  Call before any GPU work (HIP's runtime
    threads inherit the affinity).  Defaults: LOCAL_RANK / LOCAL_WORLD_SIZE from torchrun.
    When this process sees fewer GPUs than there are ranks (one GPU modelling rank 0 of a node,
    or ranks sharing GPUs), the node's full KFD GPU list stands in: rank r <-> the node's GPU r
    ("numa_source": "node_model").  Returns {"cpus", "threads", "numa", "numa_source",
    "numa_reason"} — the last says why "numa" is None."""
    lr = int(os.environ.get("LOCAL_RANK", "0")) if local_rank is None else int(local_rank)
    lw = int(os.environ.get("LOCAL_WORLD_SIZE", "1")) if local_world is None else int(local_world)
    budget = thread_budget()
    if not hasattr(os, "sched_getaffinity"):
        threads = max(1, budget // max(lw, 1))
        torch.set_num_threads(threads)
        return {"cpus": None, "threads": threads, "numa": None, "numa_source": None,
                "numa_reason": "no sched_getaffinity"}
    source, reason = None, None
    if topology == "auto":
        topo, source = host_topology(sysfs), "visible"
        if topo is None or len(topo["gpu_nodes"]) < lw:
            seen = "no KFD topology or unmappable *_VISIBLE_DEVICES" if topo is None else \
                f"{len(topo['gpu_nodes'])} visible GPU(s) for {lw} ranks"
            node = host_topology(sysfs, visible_only=False)
            if node is not None and len(node["gpu_nodes"]) >= lw:
                topo, source = node, "node_model"
            else:
                topo, source = None, None
                reason = seen + ("" if node is None else f"; the KFD lists {len(node['gpu_nodes'])} GPU(s)")
    else:
        topo, source = topology, ("given" if topology else None)
        reason = None if topology else "topology disabled"
    aff = os.sched_getaffinity(0)
    mine = rank_cpus_numa(aff, lr, lw, topo)
    numa = None
    if topo and len(topo["gpu_nodes"]) > lr and set(mine) <= set(topo["node_cpus"].get(topo["gpu_nodes"][lr], [])):
        numa = topo["gpu_nodes"][lr]
    elif topo:
        reason = "the process affinity misses a rank's NUMA node: plain slices"
    if numa is None:
        source = None
    if mine:
        os.sched_setaffinity(0, mine)
    threads = max(1, min(len(mine) or 1, budget // max(lw, 1)))
    torch.set_num_threads(threads)
    return {"cpus": mine, "threads": threads, "numa": numa, "numa_source": source, "numa_reason": reason}


def lpt_plan(durations: Sequence[float], worlds=(1, 2, 4, 8)) -> dict:
    """Predicted load balance of shard_files: max / mean rank load per world size (the
    strong-scaling ceiling of a per-file corpus run is world / (max/mean))."""
    out = {}
    for w in worlds:
        loads = [sum(float(durations[i]) for i in s) for s in shard_files(durations, w)]
        mean = sum(loads) / w
        out[str(w)] = {"max_over_mean": max(loads) / mean if mean > 0 else 1.0,
                       "max_load_s": max(loads), "ideal_speedup": w / (max(loads) / mean) if mean > 0 else float(w)}
    return out


def _encode_dictionary(d: Dict[str, int]) -> torch.Tensor:
    """[n_entries, 2 + L] int32: (id, n_codepoints, codepoints..., 0-padded)."""
    items = sorted(d.items(), key=lambda kv: (kv[1], kv[0]))
    L = max((len(k) for k, _ in items), default=0)
    t = torch.zeros((len(items), 2 + L), dtype=torch.int32)
    for r, (k, v) in enumerate(items):
        t[r, 0] = int(v)
        t[r, 1] = len(k)
        for c, ch in enumerate(k):
            t[r, 2 + c] = ord(ch)
    return t


def _decode_dictionary(t: torch.Tensor) -> Dict[str, int]:
    out = {}
    for row in t.tolist():
        n = row[1]
        out["".join(chr(c) for c in row[2:2 + n])] = row[0]
    return out


def broadcast_dictionary(dictionary: Optional[Dict[str, int]], device=None, src: int = 0,
                         force: bool = False) -> Dict[str, int]:
    """Broadcast rank `src`'s {char: id} vocabulary to every rank (two broadcasts: shape,
    then the packed table).  Device tensors for RCCL, CPU tensors for gloo.  A world of one
    returns a copy without a collective unless `force` (the RCCL test drives the device path
    on a one-GPU box that way)."""
    if not dist.is_initialized() or (dist.get_world_size() == 1 and not force):
        return dict(dictionary)
    backend = dist.get_backend()
    dev = torch.device(device) if (device is not None and backend != "gloo") else torch.device("cpu")
    if dist.get_rank() == src:
        packed = _encode_dictionary(dictionary)
        shape = torch.tensor(list(packed.shape), dtype=torch.int64)
    else:
        packed = None
        shape = torch.zeros(2, dtype=torch.int64)
    shape = shape.to(dev)
    dist.broadcast(shape, src)
    if packed is None:
        packed = torch.zeros(tuple(int(x) for x in shape.tolist()), dtype=torch.int32)
    packed = packed.to(dev)
    dist.broadcast(packed, src)
    return _decode_dictionary(packed.cpu())


def gather_results(local: Dict[int, dict], dst: int = 0) -> Optional[Dict[int, dict]]:
    """Collect {file_index: result} from every rank on `dst` (None elsewhere)."""
    if not dist.is_initialized() or dist.get_world_size() == 1:
        return dict(local)
    bucket = [None] * dist.get_world_size() if dist.get_rank() == dst else None
    dist.gather_object(local, bucket, dst=dst)
    if dist.get_rank() != dst:
        return None
    merged: Dict[int, dict] = {}
    for part in bucket:
        merged.update(part)
    return dict(sorted(merged.items()))


def align_corpus(files, align_fn, durations: Sequence[float], gather: bool = True):
    """Run align_fn(file) for this rank's share of `files`; optionally gather to rank 0.
    `align_fn` is the per-file pipeline (e.g. VAD merge_chunks -> ASR segments -> align)."""
    world = dist.get_world_size() if dist.is_initialized() else 1
    rank = dist.get_rank() if dist.is_initialized() else 0
    mine = shard_files(durations, world)[rank]
    local = {i: align_fn(files[i]) for i in mine}
    return gather_results(local) if gather else local
