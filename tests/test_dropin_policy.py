"""libbine.so's default forms for the unchanged pico_core (VERDICT r5 item 4;
bine_dropin_defaults, include/bine_amd.h): the fastest bit-identical forms by
default -- flat reduce-scatter, flat allgather and, at P > 1, the direct
peer-memory transport (whose fused one-launch form C1 and C3 take) -- the
literal schedule over RCCL with BINE_LITERAL=1, one setting overridden by its
own variable.  Host only: the same function the shim calls per communicator."""
import ctypes

import pytest

import pico_amd

VARS = ("BINE_LITERAL", "BINE_FLAT_RS", "BINE_FLAT_AG", "BINE_DIRECT")


def defaults(P):
    v = [ctypes.c_int(-1) for _ in range(3)]
    assert pico_amd.lib().bine_dropin_defaults(P, *[ctypes.byref(x) for x in v]) == 0
    return tuple(x.value for x in v)   # (flat_rs, flat_ag, direct)


@pytest.fixture
def env(monkeypatch):
    for k in VARS:
        monkeypatch.delenv(k, raising=False)
    return monkeypatch


def test_default_is_flat_and_direct(env):
    for P in (2, 4, 8, 16):
        assert defaults(P) == (1, 1, 1), P
    assert defaults(1) == (1, 1, 0)   # one rank: no exchanges, no transport to set up


def test_literal_schedule_on_request(env):
    env.setenv("BINE_LITERAL", "1")
    assert defaults(4) == (0, 0, 0)
    env.setenv("BINE_DIRECT", "1")    # one setting back on top of the literal schedule
    assert defaults(4) == (0, 0, 1)
    env.setenv("BINE_LITERAL", "0")
    env.delenv("BINE_DIRECT")
    assert defaults(4) == (1, 1, 1)


def test_single_overrides(env):
    env.setenv("BINE_DIRECT", "0")
    assert defaults(8) == (1, 1, 0)    # the flat phases over RCCL P2P
    env.setenv("BINE_FLAT_AG", "2")
    assert defaults(8) == (1, 2, 0)    # allgather cut with the reduce-scatter's chunks
    env.setenv("BINE_FLAT_AG", "7")
    assert defaults(8)[1] == 2         # clamped
    env.setenv("BINE_FLAT_RS", "0")
    assert defaults(8) == (0, 2, 0)
    env.setenv("BINE_FLAT_RS", "")     # empty = unset
    assert defaults(8)[0] == 1


def test_bad_arguments():
    assert pico_amd.lib().bine_dropin_defaults(0, None, None, None) != 0
