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
