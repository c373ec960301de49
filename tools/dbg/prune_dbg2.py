"""Debug: two engines in lockstep (pruning off / on); after each advance the
pruned lattice must stay a subset of the unpruned one."""
import os, sys
import numpy as np
R = os.path.dirname(os.path.abspath(__file__)) + "/../.."
sys.path[:0] = [R + "/tests", R + "/vosk-api_amd", R + "/vosk-api_amd/tools"]
import conftest
from conftest import perturbed_stream
from lattice_util import canon_engine
import wave
os.environ["VOSK_AMD_DEC_DEBUG"] = "1"
model = conftest._make("synth", seed=7, vocab=3000, num_pdfs=2000)
w = wave.open(R + "/tests/golden/test.wav"); x = np.frombuffer(w.readframes(w.getnframes()), "<i2").astype(np.float32)
wave_ = perturbed_stream(x, 9, seconds=15.0)
from vosk import engine
E = []
for prune in ("0", "1"):
    os.environ["VOSK_AMD_DEC_PRUNE"] = prune
    e = engine.Engine(model, frames_per_chunk=51, max_streams=2, lattice=True)
    E.append((e, e.new_stream()))
for i in range(0, len(wave_), 8160):
    for e, s in E:
        e.accept(s, wave_[i:i + 8160]); e.advance([s])
    (e0, s0), (e1, s1) = E
    st = e1.decoder_state(s1)
    L0, L1 = e0.lattice(s0, False), e1.lattice(s1, False)
    t0, l0 = canon_engine(L0); t1, l1 = canon_engine(L1)
    badf = [k for k in range(len(t0)) if not (set(t1[k]) <= set(t0[k]) and set(l1[k]) <= set(l0[k]))]
    print(i // 8160, st, "bad frames", badf[:10], len(badf), flush=True)
    if badf:
        k = badf[0]
        print(" frame", k, "tokens", len(t0[k]), len(t1[k]), "links", len(l0[k]), len(l1[k]))
        print(" missing toks", list(set(t1[k]) - set(t0[k]))[:5])
        print(" extra links", list(set(l1[k]) - set(l0[k]))[:5])
        fb = L1["frame_begin"]
        print(" frame_begin around", fb[max(0,k-3):k+4])
        break
