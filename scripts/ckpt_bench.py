#!/usr/bin/env python3
"""Batch-model save + load timing at scale: a GPU table of
``--rows`` rows (random keys, random values) is saved through the native
streaming saver (device-side compaction into a pinned double-buffered ring,
native writer threads) and loaded back into a fresh BoxWrapper through the
streamed loader (memory-mapped parts walked in LOAD_CHUNK_ROWS chunks).
Reports seconds, GB/s, peak host RSS growth and HBM beyond the table, then
checks a sample of loaded rows bit-exactly.  One JSON line on stdout.

    python scripts/ckpt_bench.py --rows 1e8 --dir /tmp/pbx_ckpt
"""
import argparse
import json
import os
import resource
import shutil
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from paddlebox_amd.ops import reference as ref  # noqa: E402
from paddlebox_amd.ps import checkpoint as ckpt  # noqa: E402
from paddlebox_amd.ps.box_wrapper import BoxWrapper  # noqa: E402
from paddlebox_amd.ps.config import SparseSGDConfig  # noqa: E402
from paddlebox_amd.ps.gpu_table import GpuSparseTable  # noqa: E402


def rss_gb():
    return resource.getrusage(resource.RUSAGE_SELF).ru_maxrss / 1e6  # KB -> GB


def log(m):
    print(m, file=sys.stderr, flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=float, default=1e8)
    ap.add_argument("--dim", type=int, default=8)
    ap.add_argument("--dir", default="/tmp/pbx_ckpt")
    ap.add_argument("--chunk", type=int, default=1 << 24, help="rows per insert / fill chunk while building")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    N = int(args.rows)
    cap = int(N / 0.8) + 1
    shutil.rmtree(args.dir, ignore_errors=True)
    t0 = time.perf_counter()
    t = GpuSparseTable(args.dim, cap, dev)
    g = torch.Generator(device=dev).manual_seed(1)
    made = 0
    while made < N:
        n = min(args.chunk, N - made)
        k = torch.randint(1, 1 << 62, (n,), device=dev, generator=g)
        h = ref.mix64(k)
        t.insert_mixed(h, SparseSGDConfig(), init_embedx=True)
        made += n
        log(f"[ckpt] built {made}/{N} rows")
    rows = t.size()
    torch.cuda.synchronize()
    log(f"[ckpt] table: {rows} rows, stride {t.t.stride if hasattr(t.t, 'stride') else '?'}, "
        f"build {time.perf_counter() - t0:.1f} s")
    hbm0 = torch.cuda.memory_allocated()
    torch.cuda.reset_peak_memory_stats()
    rss0 = rss_gb()
    t1 = time.perf_counter()
    n_saved = ckpt.save_batch_model(t, args.dir, 0)
    save_s = time.perf_counter() - t1
    st = dict(ckpt.last_save_stats)
    save_hbm = (torch.cuda.max_memory_allocated() - hbm0) / 1e9
    save_rss = rss_gb() - rss0
    nbytes = sum(os.path.getsize(os.path.join(args.dir, f)) for f in os.listdir(args.dir))
    log(f"[ckpt] saved {n_saved} rows, {nbytes / 1e9:.2f} GB in {save_s:.2f} s")
    # sample for the exactness check, then free the source table
    sel = torch.randperm(rows, device=dev, generator=g)[:100000]
    k_all, v_all = t.export(True)
    ks, vs = k_all[sel].clone(), v_all[sel].clone()
    del k_all, v_all, t
    torch.cuda.empty_cache()
    BoxWrapper._instance = None
    box = BoxWrapper(args.dim, device=dev)
    box.initialize_gpu_and_load_model(slot_vector=[1], max_keys=1 << 16, capacity=cap)
    hbm1 = torch.cuda.memory_allocated()
    torch.cuda.reset_peak_memory_stats()
    rss1 = rss_gb()
    t2 = time.perf_counter()
    n_loaded = box.load_model(args.dir)
    torch.cuda.synchronize()
    load_s = time.perf_counter() - t2
    load_hbm = (torch.cuda.max_memory_allocated() - hbm1) / 1e9
    load_rss = rss_gb() - rss1
    got = box.engine.table.read(ks)
    ok = bool(torch.equal(got[:, :vs.shape[1]], vs))
    log(f"[ckpt] loaded {n_loaded} rows in {load_s:.2f} s; sample exact: {ok}")
    out = dict(rows=rows, dim=args.dim, file_gb=round(nbytes / 1e9, 3), save_s=round(save_s, 3),
               save_gb_per_s=round(nbytes / 1e9 / save_s, 2), save_stats={k: (round(v, 3) if isinstance(v, float) else v)
                                                                          for k, v in st.items()},
               save_extra_hbm_gb=round(save_hbm, 3), save_host_rss_growth_gb=round(save_rss, 3),
               load_s=round(load_s, 3), load_gb_per_s=round(nbytes / 1e9 / load_s, 2),
               load_extra_hbm_gb=round(load_hbm, 3), load_host_rss_growth_gb=round(load_rss, 3),
               load_chunk_rows=ckpt.LOAD_CHUNK_ROWS, sample_rows_exact=ok, n_saved=n_saved, n_loaded=n_loaded)
    print(json.dumps(out), flush=True)
    shutil.rmtree(args.dir, ignore_errors=True)


if __name__ == "__main__":
    main()
