"""The reply demuxer (state_machine.Demuxer), as the reference's own property test
(src/state_machine.zig:2577-2619): random sparse replies over a full message, cut
into events of random strides; every demuxed result belongs to its range."""
import numpy as np

from tigerbeetle_amd.state_machine import Demuxer
from tigerbeetle_amd.types import RESULT_DTYPE

MESSAGE_BODY_SIZE_MAX = (1 << 20) - 256


def test_demuxer_random_strides():
    rng = np.random.default_rng(42)
    cap = MESSAGE_BODY_SIZE_MAX // RESULT_DTYPE.itemsize
    for _ in range(100):
        idx = np.nonzero(rng.random(cap) < 0.5)[0].astype(np.uint32)
        reply = np.zeros(len(idx), dtype=RESULT_DTYPE)
        reply["index"] = idx
        d = Demuxer(reply)
        event_count = max(1, int(rng.integers(0, cap + 1)))
        off, seen = 0, 0
        while off < event_count:
            size = max(1, int(rng.integers(0, event_count - off + 1)))
            got = d.decode(off, size)
            assert np.all(got["result"] == 0)
            assert np.all(got["index"] < size)
            # exactly the results whose original index fell in [off, off + size)
            want = idx[(idx >= off) & (idx < off + size)] - off
            assert np.array_equal(got["index"], want)
            seen += len(got)
            off += size
        assert seen == int(np.sum(idx < event_count))
