"""Registered GpuModels (include/stateright_gpu.h SR_MODEL_*), named after the reference models.

Each class carries the reference model's parameters and returns a `CheckerBuilder` from
`checker()`, like `Model::checker` (src/lib.rs:231-236).
"""
from . import _native as N
from .checker import CheckerBuilder


class _Model:
    MODEL_ID = 0

    def params(self):
        return []

    def checker(self):
        return CheckerBuilder(self)


class LinearEquation(_Model):
    """`LinearEquation { a, b, c }` (src/test_util.rs:140-188): find x, y with a*x + b*y == c in u8."""
    MODEL_ID = N.SR_MODEL_LINEAR_EQUATION

    def __init__(self, a, b, c):
        self.a, self.b, self.c = a, b, c

    def params(self):
        return [self.a, self.b, self.c]


class BinaryClock(_Model):
    """`BinaryClock` (src/test_util.rs:4-45)."""
    MODEL_ID = N.SR_MODEL_BINARY_CLOCK


class TwoPhaseSys(_Model):
    """`TwoPhaseSys { rms: 0..rm_count }` (examples/2pc.rs:10-121)."""
    MODEL_ID = N.SR_MODEL_2PC

    def __init__(self, rm_count):
        self.rm_count = rm_count

    def params(self):
        return [self.rm_count]


class Increment(_Model):
    """`increment` example `State::new(n)` (examples/increment.rs:109-197)."""
    MODEL_ID = N.SR_MODEL_INCREMENT

    def __init__(self, thread_count):
        self.thread_count = thread_count

    def params(self):
        return [self.thread_count]


class IncrementLock(_Model):
    """`increment_lock` example `State::new(n)` (examples/increment_lock.rs:3-107)."""
    MODEL_ID = N.SR_MODEL_INCREMENT_LOCK

    def __init__(self, thread_count):
        self.thread_count = thread_count

    def params(self):
        return [self.thread_count]


class Paxos(_Model):
    """The paxos example: `PaxosModelCfg { client_count, server_count: 3, network }` with an
    unordered non-duplicating network (examples/paxos.rs:223-263), checked through ActorModel
    (src/actor/model.rs:176-327) with a linearizability history (src/actor/register.rs:37-87).

    Action ids are canonical envelope codes (oracle/paxos.hpp `envelope_code`), so a path is
    comparable with the CPU oracle's. client_count 1..6 (the reference's bench.sh checks 6); the
    linearizability history is kept in the state and checked on the device (csrc/paxos.hpp)."""
    MODEL_ID = N.SR_MODEL_PAXOS

    def __init__(self, client_count=2, server_count=3):
        if server_count != 3:
            raise ValueError("the paxos encoding is compiled for server_count = 3 (examples/paxos.rs:275)")
        self.client_count = client_count
        self.server_count = server_count

    def params(self):
        return [self.client_count]

    KINDS = ("Prepare", "Prepared", "Accept", "Accepted", "Decided", "Put", "Get", "PutOk", "GetOk")

    @staticmethod
    def deliver(src, dst, kind, *fields):
        """Action id of `Deliver { src, dst, msg }` (src/actor/model.rs:18-24) in the canonical
        envelope code (oracle/paxos.hpp `envelope_code`). `fields` follow the reference message:
        Put(req, value), Get(req), PutOk(req), GetOk(req, value), Prepare(ballot),
        Prepared(ballot, last_accepted), Accept(ballot, proposal), Accepted(ballot),
        Decided(ballot, proposal); ballot = (round, id), proposal = (req, requester, value),
        last_accepted = None or (ballot, proposal)."""
        k = Paxos.KINDS.index(kind)

        def bal(b):
            return b[0] * 8 + b[1]

        def acc(a):
            return 0 if a is None else 1 + a[0][0] * 64 + a[0][1] * 8 + a[1][1]

        def ch(v):
            return ord(v) if isinstance(v, str) else int(v)

        if kind in ("Prepare", "Accepted"):
            f = bal(fields[0])
        elif kind == "Prepared":
            f = bal(fields[0]) * 4096 + acc(fields[1])
        elif kind in ("Accept", "Decided"):
            f = bal(fields[0]) * 16 + fields[1][1]
        elif kind in ("Put", "Get", "PutOk"):
            f = fields[0]
        else:
            f = fields[0] * 256 + ch(fields[1])
        return (((f * 16) + k) * 16 + dst) * 16 + src


class DGraph(_Model):
    """The reference's `DGraph` test fixture (src/test_util.rs:47-116): a directed graph over u8
    states built from paths, with one property "odd" (s % 2 == 1) of the given expectation — the
    model the reference checks `eventually` properties with (src/checker.rs:349-414)."""
    MODEL_ID = N.SR_MODEL_DGRAPH

    def __init__(self, expectation=N.SR_EVENTUALLY, paths=()):
        self.expectation = int(expectation)
        self.paths = [list(p) for p in paths]

    @classmethod
    def with_property(cls, expectation):
        return cls(expectation)

    def with_path(self, path):
        """`DGraph::with_path`: adds path[0] to the init states and the path's edges."""
        return DGraph(self.expectation, self.paths + [list(path)])

    def params(self):
        p = [self.expectation]
        for path in self.paths:
            p.append(len(path))
            p.extend(path)
        return p


class PingPong(_Model):
    """The reference's ping-pong actor fixture `PingPongCfg { max_nat, maintains_history }
    .into_model()` (src/actor/actor_test_util.rs:4-96) with `.lossy_network(..)` and
    `.duplicating_network(..)` (src/actor/model.rs:52-66; the reference defaults to a lossless
    duplicating network). Action ids: Deliver = envelope code * 4 + 1, Drop = code * 4 + 2
    (stateright_amd/csrc/actor.hpp). `max_nat` <= 7 runs on a 16-slot network encoding, 8..=14 on a
    32-slot one (its states describe 32 envelopes instead of 16)."""
    MODEL_ID = N.SR_MODEL_PINGPONG

    def __init__(self, max_nat, maintains_history=False, lossy=False, duplicating=True):
        self.max_nat, self.maintains_history = max_nat, maintains_history
        self.lossy, self.duplicating = lossy, duplicating

    def lossy_network(self, on=True):
        return PingPong(self.max_nat, self.maintains_history, on, self.duplicating)

    def duplicating_network(self, on=True):
        return PingPong(self.max_nat, self.maintains_history, self.lossy, on)

    def params(self):
        return [self.max_nat, int(self.lossy), int(self.duplicating), int(self.maintains_history)]


class ActorFixture(_Model):
    """The reference's one-actor fixtures (src/actor/model.rs:697-733): kind 0 =
    `handles_undeliverable_messages` (an init envelope to Id 99), kind 1 = `resets_timer`."""
    MODEL_ID = N.SR_MODEL_ACTOR_FIXTURE

    def __init__(self, kind):
        self.kind = kind

    def params(self):
        return [self.kind]


class SingleCopyRegister(_Model):
    """The single-copy register `SingleCopyModelCfg { client_count, server_count }.into_model()`
    (examples/single-copy-register.rs:40-78): SingleCopyActor servers (a register value each, no
    consensus), RegisterActor clients, a non-duplicating network and a linearizability history.
    Its `check` CLI uses one server (linearizable); two or more are not linearizable."""
    MODEL_ID = N.SR_MODEL_SINGLE_COPY

    def __init__(self, client_count=2, server_count=1):
        self.client_count, self.server_count = client_count, server_count

    def params(self):
        return [self.client_count, self.server_count]


class AbdRegister(_Model):
    """The ABD linearizable register `AbdModelCfg { client_count, server_count }.into_model()`
    (examples/linearizable-register.rs:192-229): AbdActor servers, RegisterActor clients, a
    non-duplicating network and a linearizability history."""
    MODEL_ID = N.SR_MODEL_ABD

    def __init__(self, client_count=2, server_count=2):
        self.client_count, self.server_count = client_count, server_count

    def params(self):
        return [self.client_count, self.server_count]
