#!/usr/bin/env python3
"""Extract the recorded Vosk outputs from the reference's colab notebook
(python/example/colab/vosk.ipynb, vosk 0.3.43 + vosk-model-small-en-us-0.15 on
python/example/test.wav, 4000-frame chunks) into a JSON fixture.

Run in the build container (the reference is not available on the GPU box);
the fixture (data only) is committed next to this script.
"""
import ast
import hashlib
import json
import os
import sys

REF = os.environ.get("VOSK_REFERENCE", "/root/reference")
NB = os.path.join(REF, "python", "example", "colab", "vosk.ipynb")
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "notebook_small_en_us.json")


def split_json_objects(text):
    """Split concatenated pretty-printed JSON objects."""
    objs, raws, depth, start = [], [], 0, None
    for i, ch in enumerate(text):
        if ch == "{":
            if depth == 0:
                start = i
            depth += 1
        elif ch == "}":
            depth -= 1
            if depth == 0 and start is not None:
                seg = text[start:i + 1]
                raws.append(seg)
                try:
                    objs.append(json.loads(seg))
                except json.JSONDecodeError:
                    try:  # printed Python dict repr (literal only, nothing executed)
                        objs.append(ast.literal_eval(seg))
                    except (ValueError, SyntaxError):
                        objs.append({"unparsed": seg})
                start = None
    return objs, raws


def main():
    nb = json.load(open(NB))
    cells = []
    for c in nb["cells"]:
        if c["cell_type"] != "code":
            continue
        src = "".join(c["source"])
        out = "".join("".join(o.get("text", [])) for o in c.get("outputs", []))
        if "AcceptWaveform" in src or "FinalResult" in src:
            objs, raws = split_json_objects(out) if "{" in out else ([], [])
            cells.append({"source": src, "outputs": objs, "raw_objects": raws})
    wav = os.path.join(os.path.dirname(os.path.abspath(__file__)), "test.wav")
    fixture = {
        "source": "python/example/colab/vosk.ipynb (vosk 0.3.43, vosk-model-small-en-us-0.15)",
        "test_wav_sha256": hashlib.sha256(open(wav, "rb").read()).hexdigest(),
        "chunk_frames": 4000,
        "runs": cells,
    }
    json.dump(fixture, open(OUT, "w"), indent=1)
    print(f"wrote {OUT}: {len(cells)} runs")


if __name__ == "__main__":
    sys.exit(main())
