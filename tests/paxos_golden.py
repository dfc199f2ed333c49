"""The reference's paxos discovery path (examples/paxos.rs:276-285) as canonical action ids.

Each step is `Deliver { src, dst, msg }` encoded by `Paxos.deliver` (oracle/paxos.hpp
`envelope_code`), written field by field like the reference test.
"""


def _deliver(src, dst, kind, *fields):
    # Same encoding as stateright_amd.models.Paxos.deliver, restated so the CPU-only oracle tests
    # do not depend on the product package.
    kinds = ("Prepare", "Prepared", "Accept", "Accepted", "Decided", "Put", "Get", "PutOk", "GetOk")

    def bal(b):
        return b[0] * 8 + b[1]

    def acc(a):
        return 0 if a is None else 1 + a[0][0] * 64 + a[0][1] * 8 + a[1][1]

    if kind in ("Prepare", "Accepted"):
        f = bal(fields[0])
    elif kind == "Prepared":
        f = bal(fields[0]) * 4096 + acc(fields[1])
    elif kind in ("Accept", "Decided"):
        f = bal(fields[0]) * 16 + fields[1][1]
    elif kind in ("Put", "Get", "PutOk"):
        f = fields[0]
    else:
        f = fields[0] * 256 + (ord(fields[1]) if isinstance(fields[1], str) else fields[1])
    return (((f * 16) + kinds.index(kind)) * 16 + dst) * 16 + src


PAXOS_VALUE_CHOSEN_PATH = [
    _deliver(4, 1, "Put", 4, "B"),
    _deliver(1, 0, "Prepare", (1, 1)),
    _deliver(0, 1, "Prepared", (1, 1), None),
    _deliver(1, 2, "Accept", (1, 1), (4, 4, "B")),
    _deliver(2, 1, "Accepted", (1, 1)),
    _deliver(1, 4, "PutOk", 4),
    _deliver(1, 2, "Decided", (1, 1), (4, 4, "B")),
    _deliver(4, 2, "Get", 8),
]
