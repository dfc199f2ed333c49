"""ORACLE — TEST INFRASTRUCTURE ONLY. A pure-Python restatement of the reference's single-threaded
breadth-first checker (src/checker/bfs.rs) for small models given as Python functions, and the
sliding puzzle of the reference crate's documentation (src/lib.rs:40-116), the model of the
example GpuModel plugin (examples/plugins/sliding_puzzle.hip). Pinned by that doc test: the puzzle
[1,4,2,3,5,8,6,7,0] discovers "solved" and [Down, Right, Down, Right] is a valid discovery
(src/lib.rs:89-115). No product path imports this file.
"""
from collections import deque

ALWAYS, EVENTUALLY, SOMETIMES = 0, 1, 2


def bfs(init_states, actions, next_state, properties, within_boundary=lambda s: True):
    """bfs.rs:36-342 with thread_count = 1: init states filtered by the boundary and queued in init
    order, popped from the back with successors pushed to the front (FIFO); properties evaluated
    at pop (always: discovery when the condition fails; sometimes: when it holds); a pop finding
    every property discovered stops; `generated` keeps the first generator (parent) of every state.
    Returns dict(unique, state_count, discoveries={name: [states...]}, visits=[states])."""
    inits = [s for s in init_states if within_boundary(s)]
    generated = {}
    depth = {}
    for s in inits:
        generated.setdefault(s, None)
        depth.setdefault(s, 0)
    state_count = len(inits)
    pending = deque(inits)  # pop from the back, push to the front (bfs.rs:61-66,183,263)
    discoveries = {}
    visits = []
    while pending:
        s = pending.pop()
        visits.append(s)
        awaiting = False
        for name, exp, cond in properties:
            if name in discoveries:
                continue
            if exp == ALWAYS and not cond(s):
                discoveries[name] = s
            elif exp == SOMETIMES and cond(s):
                discoveries[name] = s
            else:
                awaiting = True
        if not awaiting:  # bfs.rs:226 (nothing left to discover: the worker stops)
            break
        for a in actions(s):
            ns = next_state(s, a)
            if ns is None or not within_boundary(ns):
                continue
            state_count += 1
            if ns not in generated:
                generated[ns] = s
                depth[ns] = depth[s] + 1
                pending.appendleft(ns)

    def path(t):
        out = []
        while t is not None:
            out.append(t)
            t = generated[t]
        return out[::-1]

    return {"unique": len(generated), "state_count": state_count, "visits": visits,
            "max_depth": max(depth.values(), default=0),
            "discoveries": {n: path(s) for n, s in discoveries.items()}}


# ---- the sliding puzzle (src/lib.rs:43-88) ----
SLIDES = ("Down", "Up", "Right", "Left")
SOLVED = (0, 1, 2, 3, 4, 5, 6, 7, 8)


def puzzle_next(state, action):
    empty = state.index(0)
    y, x = divmod(empty, 3)
    frm = {"Down": empty - 3 if y > 0 else None, "Up": empty + 3 if y < 2 else None,
           "Right": empty - 1 if x > 0 else None, "Left": empty + 1 if x < 2 else None}[action]
    if frm is None:
        return None
    ns = list(state)
    ns[empty] = state[frm]
    ns[frm] = 0
    return tuple(ns)


def puzzle_bfs(cells):
    return bfs([tuple(cells)], lambda s: SLIDES, puzzle_next, [("solved", SOMETIMES, lambda s: s == SOLVED)])


def puzzle_replay(cells, actions):
    s = tuple(cells)
    states = [s]
    for a in actions:
        s = puzzle_next(s, a)
        if s is None:
            return None
        states.append(s)
    return states
