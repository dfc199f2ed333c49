"""Actor-model fixtures of the reference and their goldens, in the canonical description shared by
the oracle (oracle/actor.hpp) and the GPU encodings (stateright_amd/csrc/actor.hpp).

Sources (reference repository):
  ping-pong          src/actor/actor_test_util.rs:4-96, tests src/actor/model.rs:515-694
  undeliverable      src/actor/model.rs:697-707
  resets_timer       src/actor/model.rs:709-733
  Explorer status    src/checker/explorer.rs:370-416
  ABD register       examples/linearizable-register.rs:236-279
  single-copy reg.   examples/single-copy-register.rs:80-118
Model ids are shared with include/stateright_gpu.h (SR_MODEL_PINGPONG / _ACTOR_FIXTURE / _ABD /
_SINGLE_COPY).
"""
PINGPONG, ACTOR_FIXTURE, ABD, SINGLE_COPY = 9, 10, 11, 12

# ---- envelope codes: (msg code * 128 + dst) * 16 + src ---------------------------------------
def env_code(msg_code, src, dst):
    return (msg_code * 128 + dst) * 16 + src


def deliver(code):
    return code * 4 + 1


def drop(code):
    return code * 4 + 2


# ---- ping-pong ----------------------------------------------------------------------------------
def ping(v):
    return v * 2


def pong(v):
    return v * 2 + 1


def pingpong_params(max_nat, lossy, duplicating=True, maintains_history=False):
    return [max_nat, int(lossy), int(duplicating), int(maintains_history)]


def pingpong_state(actors, envelopes, history=(0, 0)):
    """Description: actor counts, history (#in, #out), timers (len, mask), 16 sorted codes."""
    net = sorted(env_code(m, s, d) for (s, d, m) in envelopes)
    return tuple(list(actors) + list(history) + [0, 0] + net + [-1] * (16 - len(net)))


# src/actor/model.rs:535-609: the 14 states of ping-pong (max_nat 1, lossy, duplicating)
PINGPONG_14 = {
    pingpong_state([0, 0], [(0, 1, ping(0))]),
    pingpong_state([0, 1], [(0, 1, ping(0)), (1, 0, pong(0))]),
    pingpong_state([1, 1], [(0, 1, ping(0)), (1, 0, pong(0)), (0, 1, ping(1))]),
    pingpong_state([0, 0], []),
    pingpong_state([0, 1], [(1, 0, pong(0))]),
    pingpong_state([0, 1], [(0, 1, ping(0))]),
    pingpong_state([0, 1], []),
    pingpong_state([1, 1], [(1, 0, pong(0)), (0, 1, ping(1))]),
    pingpong_state([1, 1], [(0, 1, ping(0)), (0, 1, ping(1))]),
    pingpong_state([1, 1], [(0, 1, ping(0)), (1, 0, pong(0))]),
    pingpong_state([1, 1], [(0, 1, ping(1))]),
    pingpong_state([1, 1], [(1, 0, pong(0))]),
    pingpong_state([1, 1], [(0, 1, ping(0))]),
    pingpong_state([1, 1], []),
}

# src/actor/model.rs:637-641: "must reach max" on a lossy network: lose the first Ping
PINGPONG_DROP_FIRST_PING = [drop(env_code(ping(0), 0, 1))]

PINGPONG_PROPS = ["delta within 1", "can reach max", "must reach max", "must exceed max", "#in <= #out",
                  "#out <= #in + 1"]

# ---- ABD register (examples/linearizable-register.rs) --------------------------------------------
A_PUT, A_GET, A_PUTOK, A_GETOK, A_QUERY, A_ACKQUERY, A_RECORD, A_ACKRECORD = range(8)


def vcode(ch):
    return 0 if ch in ("\0", 0, None) else ord(ch) - ord("A") + 1


def abd_msg(kind, req, seq=(0, 0), val="\0"):
    return ((((req * 8 + seq[0]) * 8 + seq[1]) * 8 + vcode(val)) * 8 + kind)


def abd_deliver(src, dst, msg):
    return deliver(env_code(msg, src, dst))


# examples/linearizable-register.rs:243-255 (BFS) and :265-277 (DFS): the same path
ABD_VALUE_CHOSEN_PATH = [
    abd_deliver(3, 1, abd_msg(A_PUT, 3, val="B")),
    abd_deliver(1, 0, abd_msg(A_QUERY, 3)),
    abd_deliver(0, 1, abd_msg(A_ACKQUERY, 3, (0, 0), "\0")),
    abd_deliver(1, 0, abd_msg(A_RECORD, 3, (1, 1), "B")),
    abd_deliver(0, 1, abd_msg(A_ACKRECORD, 3)),
    abd_deliver(1, 3, abd_msg(A_PUTOK, 3)),
    abd_deliver(3, 0, abd_msg(A_GET, 6)),
    abd_deliver(0, 1, abd_msg(A_QUERY, 6)),
    abd_deliver(1, 0, abd_msg(A_ACKQUERY, 6, (1, 1), "B")),
    abd_deliver(0, 1, abd_msg(A_RECORD, 6, (1, 1), "B")),
    abd_deliver(1, 0, abd_msg(A_ACKRECORD, 6)),
]
ABD_VALUE_CHOSEN_NAMES = [
    "Deliver { src: Id(3), dst: Id(1), msg: Put(3, 'B') }",
    "Deliver { src: Id(1), dst: Id(0), msg: Internal(Query(3)) }",
    "Deliver { src: Id(0), dst: Id(1), msg: Internal(AckQuery(3, (0, Id(0)), '\\u{0}')) }",
    "Deliver { src: Id(1), dst: Id(0), msg: Internal(Record(3, (1, Id(1)), 'B')) }",
    "Deliver { src: Id(0), dst: Id(1), msg: Internal(AckRecord(3)) }",
    "Deliver { src: Id(1), dst: Id(3), msg: PutOk(3) }",
    "Deliver { src: Id(3), dst: Id(0), msg: Get(6) }",
    "Deliver { src: Id(0), dst: Id(1), msg: Internal(Query(6)) }",
    "Deliver { src: Id(1), dst: Id(0), msg: Internal(AckQuery(6, (1, Id(1)), 'B')) }",
    "Deliver { src: Id(0), dst: Id(1), msg: Internal(Record(6, (1, Id(1)), 'B')) }",
    "Deliver { src: Id(1), dst: Id(0), msg: Internal(AckRecord(6)) }",
]

# ---- single-copy register (examples/single-copy-register.rs) ------------------------------------
# Its messages are ABD's Put / Get / PutOk / GetOk (abd_msg with seq (0, Id(0))).
# :91-96 (2 clients, 1 server, DFS; unique_state_count 93): "value chosen"
SINGLE_COPY_VALUE_CHOSEN_1 = [
    abd_deliver(2, 0, abd_msg(A_PUT, 2, val="B")),
    abd_deliver(0, 2, abd_msg(A_PUTOK, 2)),
    abd_deliver(2, 0, abd_msg(A_GET, 4)),
]
# :104-109 (2 clients, 2 servers, BFS): "linearizable" is violated
SINGLE_COPY_NOT_LINEARIZABLE_2 = [
    abd_deliver(3, 1, abd_msg(A_PUT, 3, val="B")),
    abd_deliver(1, 3, abd_msg(A_PUTOK, 3)),
    abd_deliver(3, 0, abd_msg(A_GET, 6)),
    abd_deliver(0, 3, abd_msg(A_GETOK, 6, val="\0")),
]
# :110-115: "value chosen"
SINGLE_COPY_VALUE_CHOSEN_2 = [
    abd_deliver(3, 1, abd_msg(A_PUT, 3, val="B")),
    abd_deliver(1, 3, abd_msg(A_PUTOK, 3)),
    abd_deliver(2, 0, abd_msg(A_PUT, 2, val="A")),
    abd_deliver(3, 0, abd_msg(A_GET, 6)),
]
