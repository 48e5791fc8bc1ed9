"""Host batch assembly cost: native build_batch into pageable vs pinned buffers."""
import sys
import time

import torch

sys.path.insert(0, ".")
from scripts.bench_fluid import DENSE, S, build, lines_from  # noqa: E402
from paddlebox_amd.data.synthetic import CriteoSynth  # noqa: E402
import paddlebox_amd.fluid as fluid  # noqa: E402

B = 8192
synth = CriteoSynth(total_features=int(1e9), alpha=1.05, seed=11, device="cpu")
NB = 16
lines = lines_from(synth, B, NB)
main_p, startup, slots, label, dense, pred, loss = build((400, 400, 400))
ds = fluid.DatasetFactory().create_dataset("PadBoxSlotDataset")
ds.set_use_var([label] + slots + [dense])
ds.set_batch_size(B)
ds.disable_shuffle()
ds.add_lines(lines)
nat = ds._native
L = max(int(nat.batch_len(i * B, B)) for i in range(NB))
for pin in (False, True) if torch.cuda.is_available() else (False,):
    keys = torch.empty(L + 4096, dtype=torch.int64, pin_memory=pin)
    lod = torch.empty(S * (B + 1), dtype=torch.int64, pin_memory=pin)
    den = torch.empty(B, 1 + DENSE, dtype=torch.float32, pin_memory=pin)
    for _ in range(3):
        nat.build_batch_into(0, B, keys, lod, den)
    t = time.perf_counter()
    for i in range(20):
        nat.build_batch_into((i % NB) * B, B, keys, lod, den)
    print(f"pin={pin}: build_batch_into {(time.perf_counter() - t) / 20 * 1e3:.3f} ms (L={L})", flush=True)
if not torch.cuda.is_available():
    sys.exit(0)
buf = torch.empty(L + 4096, dtype=torch.int64)
pinned = torch.empty(L + 4096, dtype=torch.int64, pin_memory=True)
t = time.perf_counter()
for _ in range(20):
    pinned.copy_(buf)
print(f"pageable->pinned copy of keys {(time.perf_counter() - t) / 20 * 1e3:.3f} ms", flush=True)
import threading  # noqa: E402

from paddlebox_amd.runtime.graph_step import pack_batch  # noqa: E402
from paddlebox_amd.runtime.trainer import _GraphBatch  # noqa: E402

torch.cuda.init()
x = torch.ones(1 << 20, device="cuda")
hb = pack_batch(_GraphBatch(torch.empty(L + 4096, dtype=torch.int64), torch.empty(S * (B + 1), dtype=torch.int64),
                            torch.empty(B, 1 + DENSE, dtype=torch.float32)), pin=True)


def timed(tag):
    t = time.perf_counter()
    for i in range(20):
        nat.build_batch_into((i % NB) * B, B, hb.keys, hb.lod, hb.dense)
    print(f"{tag}: {(time.perf_counter() - t) / 20 * 1e3:.3f} ms", flush=True)


timed("after cuda init, packed pinned, main thread")
th = threading.Thread(target=timed, args=("packed pinned, worker thread",))
th.start()
th.join()
stop = False


def busy():
    while not stop:
        sum(range(1000))


b = threading.Thread(target=busy)
b.start()
timed("main thread while another python thread spins")
stop = True
b.join()
