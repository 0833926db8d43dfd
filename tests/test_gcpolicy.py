"""utils/gcpolicy.ManualGC: automatic GC off while active, periodic young-gen
collection, state restored on close."""
import gc

from tensorflow_distributed_on_gke_amd.utils.gcpolicy import ManualGC


def test_manual_gc_cycle():
    assert gc.isenabled()
    m = ManualGC(interval=3)
    try:
        assert not gc.isenabled()
        assert gc.get_freeze_count() > 0
        got = [m.step() for _ in range(7)]
        assert got == [False, False, True, False, False, True, False]
    finally:
        m.close()
    assert gc.isenabled()
    assert gc.get_freeze_count() == 0


def test_manual_gc_disabled(monkeypatch):
    monkeypatch.delenv("TDG_MANUAL_GC", raising=False)
    m = ManualGC.from_env()
    assert gc.isenabled()
    assert not m.step()
    m.close()
    assert gc.isenabled()
