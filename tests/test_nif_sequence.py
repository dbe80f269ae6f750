"""The Erlang NIF's C-ABI call sequence without Erlang:
tests/native/nif_sequence.c creates the engine and the batching aggregator, submits
publishes from 8 "scheduler" threads that each wait for their own message (enif_send is a
mailbox here), writes a second epoch through the batcher while it runs, and destroys it
with publishes still queued (all must be answered).  CPU: over a custom backend.  GPU:
over a real engine, every publish's ids checked against a C restatement of
emqx_topic:match/2 (apps/emqx/src/emqx_topic.erl:78-102)."""
import os
import subprocess

import pytest

BIN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "native", "nif_sequence")


def _run(mode):
    if not os.path.exists(BIN):
        pytest.fail("tests/native/nif_sequence not built (run __graft_entry__.build())")
    p = subprocess.run([BIN, mode], capture_output=True, text=True, timeout=100)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-2000:]
    assert "0 failures" in p.stdout, p.stdout


def test_nif_call_sequence_cpu_backend():
    _run("cpu")


@pytest.mark.gpu
def test_nif_call_sequence_engine_gpu():
    _run("gpu")
