"""Development: repeat the 64-stream large-graph decode and report the
lattice overflow bits per run (decoder_state lat_ovf)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))
import conftest  # noqa: E402


def main():
    import numpy as np
    import wave as W
    from vosk import engine
    model = conftest._make_preset("bigram_2m")
    w = W.open(os.path.join(REPO, "tests", "golden", "test.wav"), "rb")
    base = np.frombuffer(w.readframes(w.getnframes()), "<i2").astype(np.float32)
    waves = [conftest.perturbed_stream(base, 100 + i, seconds=5.0 + 0.05 * i) for i in range(64)]
    for rep in range(int(sys.argv[1]) if len(sys.argv) > 1 else 4):
        e = engine.Engine(model, frames_per_chunk=51, max_streams=64, pipeline=True, lattice=True)
        e.set_step_samples(51 * 160)
        ss = [e.new_stream() for _ in range(64)]
        for s, x in zip(ss, waves):
            e.preload(s, x, finished=True)
        while e.step(ss):
            pass
        bad = [(s, e.decoder_state(s)["lat_ovf"], e.decoder_state(s)["err"]) for s in ss
               if e.decoder_state(s)["lat_ovf"] or e.decoder_state(s)["err"]]
        print("rep", rep, "bad", bad, flush=True)
        e.close()


if __name__ == "__main__":
    main()
