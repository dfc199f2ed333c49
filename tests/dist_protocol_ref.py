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


def pipelined_bfs(n, cmin=8192, big=262144, head_max=0):
    """The PIPELINED level loop of dist.hpp (`lag_loop`): one exchange per level of fixed-capacity
    buckets whose header carries the sender's row, planned from rows read one level behind (two
    levels ahead of them), or one level ahead when the level is big. Every decision (bucket
    capacity C, look-ahead, overflow) is a function of the rows alone, so all ranks agree. Returns
    (unique, state_count, depth, visited, plan) where plan lists (level, C, overflowed); an
    overflow ends the run (the engine then restarts in the synchronous mode)."""
    rank, world = dist.get_rank(), dist.get_world_size()
    visited, frontier = set(), []
    plan = []
    growth, pair_ratio, have_rows, prev = float(min(2 + 5 * n, 32)), 0.0, False, 0
    level = 0
    if head_max:
        # replicated head (dist.hpp run_head): every rank runs the small levels alone, no exchange
        seen, cur, state_count, depth, prev_n, spp = {0}, [0], 1, 0, 1, 1.0
        while len(cur) <= head_max:
            nxt, succ = [], 0
            for s in cur:
                for t in twopc_successors(s, n):
                    succ += 1
                    if t not in seen:
                        seen.add(t)
                        nxt.append(t)
            state_count += succ
            if not nxt:
                return len(seen), state_count, depth, len([x for x in seen if owner_of(fingerprint(x), world) == rank]), plan
            spp, prev_n = succ / len(cur), len(cur)
            cur, level, depth = nxt, level + 1, level + 1
        # hand-over: owned head states visited, owned last level = first frontier
        visited = {x for x in seen if owner_of(fingerprint(x), world) == rank}
        frontier = [x for x in cur if owner_of(fingerprint(x), world) == rank]
        unique = len(seen)
        growth, have_rows, prev = len(cur) / prev_n, True, prev_n
        pair_ratio = spp / (world * world)
        n_last = [len(cur) // world + 1] * world
        n_hi = [int(n_last[0] * max(1.0, growth) * 2) + 64] * world
        caps = {level: max(cmin, int(pair_ratio * len(cur) * 1.3) + 256)}
        head_levels = level
    else:
        if owner_of(fingerprint(0), world) == rank:
            visited.add(0)
            frontier.append(0)
        roots = torch.tensor([len(frontier)], dtype=torch.int64)
        dist.all_reduce(roots)
        unique, state_count, depth = int(roots), 1, 0
        n_last = [max(1, int(roots) // world)] * world
        n_hi = [0] * world
        caps = {0: cmin}
        head_levels = 0

    def bucket_cap(ahead):
        g = growth * 1.1
        fr = 0
        for q in range(world):
            c1 = min(n_hi[q], int(n_last[q] * g) + 64) if have_rows else n_last[q]
            fr += int(c1 * g) if ahead == 2 else c1
        return max(cmin, int(pair_ratio * fr * 1.15) + 256) if have_rows else cmin

    while True:
        glob_last = sum(n_last)
        is_big = have_rows and glob_last * growth * growth >= big
        if level + 1 not in caps and not is_big:
            first_after_head = head_levels and level == head_levels
            caps[level + 1] = bucket_cap(2 if have_rows and not first_after_head else 1)
        C = caps[level]
        # expand + route into buckets of capacity C (the row rides in every bucket's header)
        buckets = [[] for _ in range(world)]
        succ, local_new = 0, []
        for s in frontier:
            for t in twopc_successors(s, n):
                succ += 1
                if t == s:
                    continue
                o = owner_of(fingerprint(t), world)
                if o == rank:
                    if t not in visited:
                        visited.add(t)
                        local_new.append(t)
                else:
                    buckets[o].append(t)
        row = [len(b) for b in buckets] + [len(frontier), succ, len(local_new)]
        send = torch.full((world, len(row) + C), -1, dtype=torch.int64)
        for q, b in enumerate(buckets):
            send[q, :len(row)] = torch.tensor(row)
            kept = b[:C]
            if kept:
                send[q, len(row):len(row) + len(kept)] = torch.tensor([x - (1 << 63) if x >= (1 << 63) else x for x in kept])
        mats = [torch.empty_like(send) for _ in range(world)]
        dist.all_gather(mats, send)  # gloo has no all_to_all: keep our column
        recv = [mats[src][rank] for src in range(world)]
        rows = [recv[src][:len(row)].tolist() for src in range(world)]
        overflow = any(rows[src][q] > C for src in range(world) for q in range(world))
        plan.append((level, C, overflow))
        if overflow:
            return unique, state_count, depth, len(visited), plan
        new = list(local_new)
        for src in range(world):
            for x in recv[src][len(row):len(row) + rows[src][rank]].tolist():
                if x not in visited:
                    visited.add(x)
                    new.append(x)
        frontier = new
        # the host reads the rows of this level
        glob_n = sum(r[world] for r in rows)
        maxpair = max(r[q] for r in rows for q in range(world))
        for q in range(world):
            n_hi[q] = rows[q][world + 2] + sum(rows[s][q] for s in range(world))
            n_last[q] = rows[q][world]
        if glob_n:
            pair_ratio = maxpair / glob_n
            if prev:
                growth = glob_n / prev
            have_rows = True
        prev = glob_n
        if glob_n == 0:
            break
        if level > head_levels:
            unique += glob_n
        depth = level
        state_count += sum(r[world + 1] for r in rows)
        if level + 1 not in caps:
            caps[level + 1] = bucket_cap(1)
        level += 1
    return unique, state_count, depth, len(visited), plan
