"""Concurrent KaldiRecognizer throughput (bench.concurrent_recognizers) for
several thread counts; for profiling the recognizer group's batched pass."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    threads = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "32").split(",")]
    seconds = float(sys.argv[2]) if len(sys.argv) > 2 else 20.0
    model = sys.argv[3] if len(sys.argv) > 3 else bench.bench_model(0, None, "la_small_en_us")
    import vosk
    vosk.SetLogLevel(-1)
    base = bench.load_wave()
    for t in threads:
        print(json.dumps(bench.concurrent_recognizers(model, base, threads=t, seconds=seconds)), flush=True)


if __name__ == "__main__":
    main()
