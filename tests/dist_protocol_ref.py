"""CPU restatement of the partitioned level loop (stateright_amd/csrc/dist.hpp) over gloo —
TEST INFRASTRUCTURE ONLY. Each rank owns the states whose fingerprint maps to it, expands its own
frontier, routes successor records to their owners (all-to-all), and the owners dedup; a row
all-gather per level carries the counts. Used to check the protocol (ownership, exchange,
termination, global totals) with world_size 2 on the CPU.
"""
import torch
import torch.distributed as dist

M64 = (1 << 64) - 1


def fmix64(k):
    k ^= k >> 33
    k = (k * 0xff51afd7ed558ccd) & M64
    k ^= k >> 33
    k = (k * 0xc4ceb9fe1a85ec53) & M64
    k ^= k >> 33
    return k


def fingerprint(packed):  # models.hpp fingerprint<1>
    return fmix64(packed ^ (1 << 63))


def owner_of(fp, nparts):  # kernels_dist.hpp owner_of
    return ((fp >> 32) * nparts) >> 32


def twopc_successors(s, n):
    """examples/2pc.rs:56-104 on the packed encoding of models.hpp TwoPhase."""
    rmask = (1 << n) - 1
    tm = (s >> (2 * n)) & 3
    prepared = (s >> (2 * n + 2)) & rmask
    msgp = (s >> (3 * n + 2)) & rmask
    commit, abort = (s >> (4 * n + 2)) & 1, (s >> (4 * n + 3)) & 1
    out = []
    if tm == 0 and prepared == rmask:
        out.append((s & ~(3 << (2 * n))) | (1 << (2 * n)) | (1 << (4 * n + 2)))
    if tm == 0:
        out.append((s & ~(3 << (2 * n))) | (2 << (2 * n)) | (1 << (4 * n + 3)))
    for rm in range(n):
        r = (s >> (2 * rm)) & 3
        clr = s & ~(3 << (2 * rm))
        if tm == 0 and (msgp >> rm) & 1:
            out.append(s | (1 << (2 * n + 2 + rm)))
        if r == 0:
            out.append(clr | (1 << (2 * rm)) | (1 << (3 * n + 2 + rm)))
            out.append(clr | (3 << (2 * rm)))
        if commit:
            out.append(clr | (2 << (2 * rm)))
        if abort:
            out.append(clr | (3 << (2 * rm)))
    return out


def partitioned_bfs(n):
    """Runs on every rank of an initialised gloo group; returns (unique, state_count, depth)."""
    rank, world = dist.get_rank(), dist.get_world_size()
    visited = set()
    init = 0
    frontier = []
    roots = 0
    if owner_of(fingerprint(init), world) == rank:
        visited.add(init)
        frontier.append(init)
        roots = 1
    unique = torch.tensor([roots], dtype=torch.int64)
    dist.all_reduce(unique)
    unique = int(unique)
    state_count, depth, level = 1, 0, 0
    while True:
        # 1. expand + route
        buckets = [[] for _ in range(world)]
        succ = 0
        local_new = []
        for s in frontier:
            for t in twopc_successors(s, n):
                succ += 1
                if t == s:
                    continue  # self-loop: counted, never routed
                o = owner_of(fingerprint(t), world)
                if o == rank:
                    if t not in visited:
                        visited.add(t)
                        local_new.append(t)
                else:
                    buckets[o].append(t)
        # 2. row all-gather: [sends per destination..., frontier size, successors]
        row = torch.tensor([len(b) for b in buckets] + [len(frontier), succ], dtype=torch.int64)
        rows = [torch.zeros_like(row) for _ in range(world)]
        dist.all_gather(rows, row)
        glob_n = sum(int(r[world]) for r in rows)
        if glob_n == 0:
            break
        if level > 0:
            unique += glob_n
        depth = level
        state_count += sum(int(r[world + 1]) for r in rows)
        # 3. all-to-all of the records (padded tensors)
        width = max(int(r[q]) for r in rows for q in range(world)) or 1
        send = torch.full((world, width), -1, dtype=torch.int64)
        for q, b in enumerate(buckets):
            if b:
                send[q, :len(b)] = torch.tensor([x - (1 << 63) if x >= (1 << 63) else x for x in b])
        # gloo has no all_to_all: all-gather every rank's send matrix and keep our column
        mats = [torch.empty_like(send) for _ in range(world)]
        dist.all_gather(mats, send)
        recv = [mats[src][rank] for src in range(world)]
        # 4. owners insert
        new = list(local_new)
        for src in range(world):
            for x in recv[src][: int(rows[src][rank])].tolist():
                if x not in visited:
                    visited.add(x)
                    new.append(x)
        frontier = new
        level += 1
    return unique, state_count, depth, len(visited)
