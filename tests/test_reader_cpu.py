"""Host logic of the reader mirror that needs no GPU: RowGroupPipeline releases the
contexts it already created when a later one fails, and the device error is what surfaces."""
import pytest

from pfloor import reader as R


class _FakeDec:
    made, closed = [], []

    def __init__(self, device=None, share=None):
        if share is not None and len(_FakeDec.made) >= 2:
            raise RuntimeError("hipErrorOutOfMemory (fake)")
        _FakeDec.made.append(self)

    def close(self):
        _FakeDec.closed.append(self)

    def wait(self):
        return 0


def test_pipeline_init_failure_closes_partial_slots(monkeypatch):
    _FakeDec.made, _FakeDec.closed = [], []
    monkeypatch.setattr(R, "GpuDecoder", _FakeDec)
    with pytest.raises(RuntimeError, match="fake"):
        R.RowGroupPipeline(None, [], [0, 1], devices=(0, 1), depth=2)
    # device 0: owner + twin; device 1: the owner was created, its twin failed
    assert len(_FakeDec.made) == 3
    assert sorted(map(id, _FakeDec.closed)) == sorted(map(id, _FakeDec.made))


def test_pipeline_rejects_empty_devices():
    with pytest.raises(ValueError):
        R.RowGroupPipeline(None, [], [0], devices=())
