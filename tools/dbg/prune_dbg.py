"""Debug: streaming engine lattice with / without pruning, frame by frame."""
import os, sys
import numpy as np
R = os.path.dirname(os.path.abspath(__file__)) + "/../.."
sys.path[:0] = [R + "/tests", R + "/vosk-api_amd", R + "/vosk-api_amd/tools"]
import conftest
from conftest import perturbed_stream
from lattice_util import canon_engine
import oracle_py
import wave
model = conftest._make("synth", seed=7, vocab=3000, num_pdfs=2000)
w = wave.open(R + "/tests/golden/test.wav"); x = np.frombuffer(w.readframes(w.getnframes()), "<i2").astype(np.float32)
wave_ = perturbed_stream(x, 9, seconds=float(sys.argv[1]) if len(sys.argv) > 1 else 15.0)
from vosk import engine
o = oracle_py.OracleModel(model, fpc=51)
res = {}
for prune in ("0", "1"):
    os.environ["VOSK_AMD_DEC_PRUNE"] = prune
    e = engine.Engine(model, frames_per_chunk=51, max_streams=2, lattice=True)
    s = e.new_stream()
    states = []
    for i in range(0, len(wave_), 8160):
        e.accept(s, wave_[i:i + 8160]); e.advance([s]); states.append(e.decoder_state(s))
    e.accept(s, np.zeros(0, np.float32), finished=True); e.advance([s])
    L = e.lattice(s, use_final=False)
    res[prune] = (L, canon_engine(L), states, e.best_path(s, use_final=False))
    print(prune, e.decoder_state(s))
for st in res["1"][2][:12]: print(st)
t0, l0 = res["0"][1]; t1, l1 = res["1"][1]
bad = 0
for k in range(len(t0)):
    a = set(t1[k]) <= set(t0[k]); b = set(l1[k]) <= set(l0[k])
    if not (a and b) or k < 3:
        print("frame", k, "tok", len(t0[k]), len(t1[k]), a, "links", len(l0[k]), len(l1[k]), b)
        bad += 1
        if bad > 8: break
print("paths equal", np.array_equal(res["0"][3][0], res["1"][3][0]))
w0 = engine.lattice_words(res["0"][0], o.graph.ilabel, o.graph.olabel, 6.0, 0.9, 5)
w1 = engine.lattice_words(res["1"][0], o.graph.ilabel, o.graph.olabel, 6.0, 0.9, 5)
print({k: (w0[k], w1[k]) for k in w0 if k not in ("nbest", "mbr") and w0[k] != w1[k]})
