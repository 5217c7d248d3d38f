"""Host CPU budget of one rank (self-play's native engine threads, Coach.py:95-100 sharded over
one process per GPU): how many cores this process may use, how many engine threads each rank
gets, and pinning a rank to the NUMA node of its GPU.

Everything here is best effort and reads only sysfs / the affinity mask: a missing file leaves
the process as it was.  pin_rank_to_gpu_numa must run before the process touches the GPU
(torch.cuda / HIP), so later threads -- the engine's OpenMP pool -- inherit the mask; it never
re-executes the process."""
import os


def _read(path):
    try:
        with open(path) as f:
            return f.read().strip()
    except OSError:
        return None


def cgroup_cpu_quota():
    """CPUs granted by a cgroup CPU quota (v2 cpu.max or v1 cfs), or None when unlimited."""
    v = _read("/sys/fs/cgroup/cpu.max")
    if v:
        a, _, b = v.partition(" ")
        if a != "max":
            try:
                return max(1, int(int(a) / int(b or 100000)))
            except ValueError:
                pass
    q, p = _read("/sys/fs/cgroup/cpu/cpu.cfs_quota_us"), _read("/sys/fs/cgroup/cpu/cpu.cfs_period_us")
    try:
        if q and p and int(q) > 0:
            return max(1, int(int(q) / int(p)))
    except ValueError:
        pass
    return None


# True when engine_omp_defaults set OMP_WAIT_POLICY (the CPU baselines' child drops it again)
_SET_WAIT_POLICY = False


def engine_omp_defaults():
    """OpenMP settings for the self-play engine's thread pool, set only where the user set
    nothing, and only effective before the OpenMP runtime starts (call before importing torch):
    OMP_WAIT_POLICY=PASSIVE -- idle workers sleep instead of spinning between the engine's
    parallel regions.  Measured on the GPU box (profiles/r04i/spwait_ab.jsonl): the self-play leg
    used 90 CPU-s and was throttled by the 16-CPU cgroup quota in ~35 of ~70 periods with
    spinning workers, 35 CPU-s and never throttled with sleeping ones, at the same games/s --
    cores another rank of the node can use."""
    global _SET_WAIT_POLICY
    if "OMP_WAIT_POLICY" not in os.environ:
        os.environ["OMP_WAIT_POLICY"] = "PASSIVE"
        _SET_WAIT_POLICY = True


def cgroup_cpu_stat():
    """The cgroup's CPU accounting (v2 cpu.stat: usage_usec, nr_periods, nr_throttled,
    throttled_usec ...) as ints, {} when not readable.  Deltas around a run show whether a CPU
    quota throttled it (every thread of the cgroup stops for the rest of a period once the
    quota is spent)."""
    out = {}
    for line in (_read("/sys/fs/cgroup/cpu.stat") or "").splitlines():
        k, _, v = line.partition(" ")
        try:
            out[k] = int(v)
        except ValueError:
            pass
    return out


def affinity():
    try:
        return sorted(os.sched_getaffinity(0))
    except AttributeError:            # pragma: no cover (non-Linux)
        return list(range(os.cpu_count() or 1))


def host_cpus():
    """Cores this process may run on: its affinity mask, capped by a cgroup CPU quota."""
    n = len(affinity())
    q = cgroup_cpu_quota()
    return min(n, q) if q else n


def local_world_size():
    try:
        return max(1, int(os.environ.get("LOCAL_WORLD_SIZE", "1") or 1))
    except ValueError:
        return 1


# True once pin_rank_to_gpu_numa has narrowed this process's affinity mask to the rank's own share
# of the cores: the mask is then per rank, and only node-wide limits are split among the ranks.
_MASK_PER_RANK = False


def threads_per_rank(local_world=None, cap=16):
    """Engine threads for this rank, at most `cap` (16: on a 16-core share, 32 threads halved
    games/s, profiles/r02s_selfplay_sweep.jsonl).  The node-wide limits -- an affinity mask
    that was not narrowed per rank, a cgroup CPU quota -- are split evenly among the
    LOCAL_WORLD_SIZE ranks; a mask pin_rank_to_gpu_numa already narrowed to this rank's share
    is used as it is (dividing it again gave 8 ranks on two 64-core nodes 2 threads each)."""
    lw = local_world or local_world_size()
    n = len(affinity())
    if not _MASK_PER_RANK:
        n //= lw
    q = cgroup_cpu_quota()
    if q:
        n = min(n, q // lw)
    return max(1, min(cap, n))


def _cpulist(s):
    out = []
    for part in (s or "").split(","):
        part = part.strip()
        if not part:
            continue
        if "-" in part:
            a, b = part.split("-")
            out.extend(range(int(a), int(b) + 1))
        else:
            out.append(int(part))
    return out


def gpu_numa_nodes():
    """NUMA node of each GPU in KFD topology order (HIP's device order), from the GPU node's
    io_link to a CPU node; None entries where sysfs does not say."""
    root = "/sys/class/kfd/kfd/topology/nodes"
    try:
        ids = sorted(int(d) for d in os.listdir(root) if d.isdigit())
    except OSError:
        return []
    cpu_nodes, gpus = [], []
    for i in ids:
        props = {}
        for line in (_read(f"{root}/{i}/properties") or "").splitlines():
            k, _, v = line.partition(" ")
            props[k] = v
        simd = int(props.get("simd_count", "0") or 0)
        if simd > 0:
            gpus.append(i)
        elif int(props.get("cpu_cores_count", "0") or 0) > 0:
            cpu_nodes.append(i)
    out = []
    for g in gpus:
        numa = None
        links = f"{root}/{g}/io_links"
        try:
            for l in sorted(os.listdir(links)):
                for line in (_read(f"{links}/{l}/properties") or "").splitlines():
                    k, _, v = line.partition(" ")
                    if k == "node_to" and int(v) in cpu_nodes:
                        numa = cpu_nodes.index(int(v))
                if numa is not None:
                    break
        except OSError:
            pass
        out.append(numa)
    return out


def pin_rank_to_gpu_numa(local_rank, local_world=None):
    """Restrict this process to the CPUs of its GPU's NUMA node (this rank's even share of them
    when several local ranks' GPUs sit on that node), intersected with the current mask.
    Returns what was done: {"numa_node", "cpus", "pinned"}."""
    lw = local_world or local_world_size()
    numas = gpu_numa_nodes()
    vis = os.environ.get("HIP_VISIBLE_DEVICES") or os.environ.get("ROCR_VISIBLE_DEVICES")
    order = list(range(len(numas)))
    if vis:
        try:
            order = [int(v) for v in vis.split(",") if v.strip() != ""]
        except ValueError:
            pass
    info = {"numa_node": None, "cpus": len(affinity()), "pinned": False}
    if local_rank >= len(order) or order[local_rank] >= len(numas):
        return info
    node = numas[order[local_rank]]
    if node is None:
        return info
    info["numa_node"] = node
    allowed = set(affinity())
    cpus = [c for c in _cpulist(_read(f"/sys/devices/system/node/node{node}/cpulist"))
            if c in allowed]
    if not cpus:
        return info
    peers = [r for r in range(min(lw, len(order)))
             if order[r] < len(numas) and numas[order[r]] == node]
    if local_rank in peers and len(peers) > 1:
        k = peers.index(local_rank)
        per = len(cpus) // len(peers)
        if per >= 1:
            cpus = cpus[k * per:(k + 1) * per]
    try:
        os.sched_setaffinity(0, cpus)
    except (AttributeError, OSError):
        return info
    global _MASK_PER_RANK
    _MASK_PER_RANK = True
    info.update(cpus=len(cpus), pinned=True)
    return info
