import os, sys
sys.path[:0] = [os.getcwd(), os.path.join(os.getcwd(), "vosk-api_amd")]
import bench
model = bench.bench_model(0, None, "la_small_en_us")
import vosk
vosk.SetLogLevel(0)
os.environ["VOSK_BATCH_MODEL_DIR"] = model
bm = vosk.BatchModel()
del bm
m = vosk.Model(model)
r = vosk.KaldiRecognizer(m, 16000)
del r, m
