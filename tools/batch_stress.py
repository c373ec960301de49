"""Development stress run of the batch path's segmentation (not a test):
decode the same streams through vosk_batch_* many times under varied lane
configurations (1 or 2 lanes on device 0, Wait() per round or everything
queued, the lane's own schedule or a seeded random one) and compare every
run with the oracle (tests/batch_expect.py).  Prints one line per run and the
full result lists of any stream that differs.

    python tools/batch_stress.py --runs 60 --out gpurun_out/stress.json
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path[:0] = [os.path.join(REPO, "tests"), os.path.join(REPO, "vosk-api_amd"),
                os.path.join(REPO, "vosk-api_amd", "tools")]

import numpy as np  # noqa: E402

import conftest  # noqa: E402
import batch_expect  # noqa: E402
from test_batching import _decode_batch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--runs", type=int, default=40)
    ap.add_argument("--streams", type=int, default=10)
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    import vosk
    vosk.SetLogLevel(-1)
    model = conftest._make("synth", seed=7, vocab=3000, num_pdfs=2000)
    ep = os.path.join(conftest.MODEL_CACHE, f"synth_ep_{conftest.SYNTH_VERSION}")
    if not os.path.exists(os.path.join(ep, "README")):
        import shutil
        tmp = ep + ".tmp"
        shutil.rmtree(tmp, ignore_errors=True)
        shutil.copytree(model, tmp)
        with open(os.path.join(tmp, "conf", "model.conf"), "a") as f:
            f.write(conftest.EP_RULES)
        os.rename(tmp, ep)
    import wave
    w = wave.open(os.path.join(REPO, "tests", "golden", "test.wav"), "rb")
    base = np.frombuffer(w.readframes(w.getnframes()), "<i2").astype(np.float32)
    waves = [conftest.perturbed_stream(base, 300 + i, seconds=5.0 + 0.9 * i) for i in range(args.streams)]
    t0 = time.time()
    exp = batch_expect.expected(ep, waves)
    print(f"oracle: {sum(len(r) for r in exp)} segments in {time.time() - t0:.1f} s", flush=True)
    os.environ["VOSK_BATCH_MODEL_DIR"] = ep
    for k in ("VOSK_AMD_DEVICE", "LOCAL_RANK"):
        os.environ.pop(k, None)
    rng = np.random.default_rng(5)
    log = []
    bad = 0
    for run in range(args.runs):
        devices = ["0", "0,0"][run % 2]
        pattern = ["wait_per_round", "queued_upfront"][(run // 2) % 2]
        seed = 0 if run % 8 < 4 else int(rng.integers(1, 1 << 30))
        os.environ["VOSK_AMD_BATCH_DEVICES"] = devices
        if seed:
            os.environ["VOSK_AMD_BATCH_SCHEDULE"] = str(seed)
        else:
            os.environ.pop("VOSK_AMD_BATCH_SCHEDULE", None)
        t1 = time.time()
        out, lanes, nl, counters = _decode_batch(vosk, waves, pattern)
        diffs = []
        for i in range(len(waves)):
            try:
                batch_expect.check(out[i], exp[i], f"stream {i}")
            except AssertionError as ex:
                diffs.append(dict(stream=i, lane=lanes[i], error=str(ex)[:400],
                                  got=[json.loads(r).get("text") for r in out[i]],
                                  got_times=[[(x["start"], x["end"]) for x in json.loads(r).get("result", [])][:1]
                                             + [(x["start"], x["end"]) for x in json.loads(r).get("result", [])][-1:]
                                             for r in out[i]],
                                  exp=[e["text"] for e in exp[i]], exp_start=[e["start"] for e in exp[i]]))
        bad += bool(diffs)
        rec = dict(run=run, devices=devices, pattern=pattern, schedule=seed, counters=counters,
                   seconds=round(time.time() - t1, 2), diffs=diffs)
        log.append(rec)
        print(json.dumps({k: rec[k] for k in ("run", "devices", "pattern", "schedule", "counters", "seconds")})
              + f" mismatching_streams={len(diffs)}", flush=True)
        for d in diffs:
            print("  MISMATCH", json.dumps(d), flush=True)
    print(f"runs {args.runs}, runs with a mismatch {bad}", flush=True)
    if args.out:
        with open(args.out, "w") as f:
            json.dump(log, f, indent=1)


if __name__ == "__main__":
    main()
