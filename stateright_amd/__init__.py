"""stateright_amd — an MI355X-native engine for Stateright's breadth-first model checker.

    from stateright_amd import TwoPhaseSys
    checker = TwoPhaseSys(9).checker().spawn_bfs().join()
    checker.assert_properties()

The hot path (frontier expansion, fingerprinting, the HBM visited set, stream compaction and
property evaluation) runs as hand-written HIP kernels for gfx950 behind the C ABI in
include/stateright_gpu.h; this package is the host-side mirror of the reference API.
"""
from .checker import CheckerBuilder, CheckerError, Expectation, GpuBfsChecker, Path, PathRecorder, StateRecorder
from .models import (AbdRegister, ActorFixture, BinaryClock, DGraph, Increment, IncrementLock, LinearEquation, Paxos,
                     PingPong, SingleCopyRegister, TwoPhaseSys)

__all__ = ["CheckerBuilder", "CheckerError", "Expectation", "GpuBfsChecker", "Path", "PathRecorder", "StateRecorder",
           "AbdRegister", "ActorFixture", "BinaryClock", "DGraph", "Increment", "IncrementLock", "LinearEquation", "Paxos",
           "PingPong", "SingleCopyRegister", "TwoPhaseSys"]
