"""The batch path's fallback words (a segment whose lattice is unusable) come
from the segment's lattice records on the host (vosk_impl.cc
SegmentBestPath); they must equal the traceback kernel's best path, with and
without final states reached, over a window that includes pruning passes."""
import numpy as np
import pytest

from conftest import perturbed_stream

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("seconds", [3.0, 9.0])
def test_segment_best_path_matches_traceback(synth_model, test_wave, seconds):
    from vosk import engine as ve
    e = ve.Engine(synth_model, frames_per_chunk=51, max_streams=4, lattice=True)
    e.set_step_samples(51 * 160)
    ss = [e.new_stream() for _ in range(4)]
    for i, s in enumerate(ss):
        e.preload(s, perturbed_stream(test_wave, 300 + i, seconds=seconds), finished=(i % 2 == 0))
    for _ in range(int(seconds * 16000 / (51 * 160)) + 4):
        if not e.step(ss):
            break
    for s in ss:
        dev, _, _ = e.best_path(s, use_final=True)
        host = e.segment_best_path(s)
        assert len(dev) > 0
        np.testing.assert_array_equal(host, dev)
    e.close()
