#!/usr/bin/env python3
"""bench.py — Mpixels/s of bit-exact HEIC decode on MI355X (BASELINE.json metric).

Workload (one shard per GPU, weak scaling): every
rank decodes a batch of `--batch` synthetic 4032x3024 8-bit 4:2:0 intra HEIC
stills; image i is halfmoonbay.heic with its 48 grid tiles permuted by
mt19937_64(seed=i) (heif_amd/synthetic.py).  A "step" is one decode of the
whole batch: bitstreams, parameter sets and slice headers are resident in HBM
before timing (host demux + upload happen once, outside the timed region);
the step runs the decode's gfx950 kernels and writes every image's cropped
Y/Cb/Cr planes to HBM.  `value` = all ranks' output luma pixels / max-over-
ranks wall time of K steps.

roofline: the dominant kernel (k_parse) measured with HIP events on the
internal parse stream it runs on, averaged over the timed steps (so the
slowdown from the overlapping reconstruction is included, as in the rocprofv3
kernel-trace average of the same command); algorithmic bytes per image =
compressed tile bytes + reconstructed planes (SURVEY.md §8(d):
1,704,187 + 18,874,368 B).

--workload config5 (side measurement, not the headline line): BASELINE
config 5, 7680x4320 Main-10 grids (15 x 9 tiles of 512x512, 16-bit planes)
from heif_amd/synth_encoder.py; image i is a permutation (seed i) of one pool
of 135 synthetic 10-bit tiles.

--split tiles (BASELINE config 5 "1->8 GPUs"): every rank
holds the SAME --batch images and decodes only the grid tiles k with
k % world == rank (heifgpu_batch_opts), so the total work is fixed
(`scaling: "strong"`) and `value` = the batch's output pixels / time.  The
gather to one device (heifgpu_gather_tiles, xGMI peer copies) is not in the
timed region.

e2e (rank 0, default on): the PCIe-inclusive rate beside `value`: the same
files re-parsed on the host (heifgpu_image_parse_many on a thread pool),
flattened into pinned memory and uploaded (heifgpu_batch_prepare_ex, two
batches reloaded alternately) while the previous batch decodes.

cpu_baseline: the CPU oracle (oracle/, spec restatement; the reference Rust
path cannot decode pixels), built -march=native on the measuring host,
decoding tiles on one thread per CPU this job may use (the cgroup quota) for
~10 s; the 1-core figure and the node's CPU count are reported beside it.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import json
import os
import pathlib
import sys
import time

ROOT = pathlib.Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

SAMPLE = ROOT / "tests" / "golden" / "halfmoonbay.heic"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md)
ROUND = "r06"
PROFILES = ROOT / "profiles" / ROUND
BINS_PER_IMAGE = 15358022  # CABAC bins of one halfmoonbay image (oracle count; every permutation has the same)


def dist_env():
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    return rank, world, local


def _free_port() -> int:
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n: int, argv: list) -> int:
    """`--gpus N` without a torchrun environment: start N copies of this
    script, one per GPU (RANK = LOCAL_RANK = r, WORLD_SIZE = N, rendezvous on
    127.0.0.1), and return a non-zero code if any rank fails.  The parent
    never imports torch or touches the GPU: it only waits, and ends the other
    ranks when one fails so none is left blocked in a collective.  Rank 0
    inherits stdout and prints the JSON line; the other ranks print nothing.
    Images (and tiles) are what shard (/root/reference/src/heic/decoder.rs:114-119),
    so there is no data-path collective to set up here."""
    import signal
    import subprocess

    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, str(pathlib.Path(__file__).resolve())] + argv, env=env))

    def _term(signum, frame):
        raise SystemExit(128 + signum)

    signal.signal(signal.SIGTERM, _term)
    rc = 0
    try:
        live = list(procs)
        while live:
            for p in list(live):
                code = p.poll()
                if code is None:
                    continue
                live.remove(p)
                if code != 0 and rc == 0:
                    rc = code if code > 0 else 128 - code
                    print(f"bench.py: rank {procs.index(p)} exited with {code}; stopping the others",
                          file=sys.stderr, flush=True)
                    for q in live:
                        q.terminate()
            time.sleep(0.05)
    finally:
        for p in procs:
            if p.poll() is None:
                p.terminate()
                try:
                    p.wait(timeout=20)
                except subprocess.TimeoutExpired:
                    p.kill()
                    p.wait()
    return rc


def dry_run(args) -> None:
    """`--dry-run`: the multi-rank skeleton of main() with no GPU (gloo):
    rendezvous, this rank's shard, barrier + timed region + MAX reduction,
    and rank 0's JSON line with `n_gpus` = world size.  Tests the launcher."""
    import torch
    import torch.distributed as dist

    rank, world, _ = dist_env()
    if os.environ.get("BENCH_DRY_FAIL_RANK") == str(rank):  # the launcher test's failing rank
        raise SystemExit(f"rank {rank}: failing on request")
    if world > 1:
        dist.init_process_group("gloo")
    seeds = shard_seeds(args.batch, rank)
    ranks = [(rank, os.getpid(), seeds)]
    if world > 1:
        ranks = [None] * world
        dist.all_gather_object(ranks, (rank, os.getpid(), seeds))
        dist.barrier()
    t0 = time.perf_counter()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed])
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    if rank == 0:
        print(json.dumps({"metric": "dry run (no GPU)", "value": None, "n_gpus": world, "steps": args.steps,
                          "warmup": args.warmup, "elapsed_s": elapsed,
                          "ranks": [{"rank": r, "pid": p, "seeds": [s[0], s[-1] + 1] if s else []}
                                    for r, p, s in ranks]}), flush=True)
    if world > 1:
        dist.destroy_process_group()


def shard_seeds(batch_per_rank: int, rank: int) -> list:
    """Image seeds of this rank: a contiguous block of the global batch."""
    return list(range(rank * batch_per_rank, (rank + 1) * batch_per_rank))


def effective_cpus() -> int:
    """CPUs this process may use: affinity mask, capped by a cgroup v2 cpu.max quota."""
    n = len(os.sched_getaffinity(0))
    try:
        quota, period = pathlib.Path("/sys/fs/cgroup/cpu.max").read_text().split()
        if quota != "max":
            n = min(n, max(1, -(-int(quota) // int(period))))
    except (OSError, ValueError):
        pass
    return n


def native_oracle() -> str:
    """Builds the oracle with -march=native for this host (oracle/Makefile
    `native`) and selects it; returns a note for the JSON line."""
    import subprocess

    try:
        subprocess.run(["make", "-s", "-C", str(ROOT / "oracle"), "native"], check=True, capture_output=True,
                       timeout=300)
    except (OSError, subprocess.SubprocessError) as e:
        return f"-O3 portable build (native build failed: {type(e).__name__})"
    if "oracle.oracle" in sys.modules:
        return "-O3 portable build (oracle already loaded)"
    os.environ["ORACLE_LIBRARY"] = str(ROOT / "oracle" / "build" / "native" / "liboracle.so")
    return "-O3 -march=native build on this host"


def cpu_baseline(data: bytes, seconds: float, threads: int, label: str = "halfmoonbay") -> dict:
    from oracle import oracle

    tiles, (ho, hl) = oracle.list_tiles(data)
    hvcc = data[ho:ho + hl]
    items = [data[o:o + n] for o, n in tiles]
    meta = oracle.read_meta(data)
    tw, th = meta["tile_width"], meta["tile_height"]
    out_px_per_tile = meta["out_width"] * meta["out_height"] / len(items)
    count = 0
    deadline = time.perf_counter() + seconds

    def worker(k):
        n = 0
        i = k
        while time.perf_counter() < deadline:
            oracle.decode_tile(hvcc, items[i % len(items)], tw, th)
            n += 1
            i += threads
        return n

    t0 = time.perf_counter()
    with cf.ThreadPoolExecutor(threads) as ex:
        count = sum(ex.map(worker, range(threads)))
    dt = time.perf_counter() - t0
    return {
        "value": round(count * out_px_per_tile / dt / 1e6, 2),
        "unit": "Mpixels/s",
        "cores": threads,
        "kind": "port",
        "sample": f"{count} {label} {tw}x{th} tiles decoded by the C oracle in {dt:.1f} s "
                  f"({threads} threads, output-pixel-equivalent of {count / len(items):.1f} "
                  f"{meta['out_width']}x{meta['out_height']} images)",
    }


def verify_images(outs, seeds, src, info, stride, offset, threads) -> int:
    """Checks every given image bit-exactly against the oracle without
    re-decoding whole images: image `seed` places tile perm_seed[k] of `src`
    (the identity-order grid) at grid position k, so each of its tile windows
    must equal the oracle's decode of that one tile of `src` (the per-tile
    loop the batch replaces, /root/reference/src/heic/decoder.rs:114-119).
    With a tile split only this rank's positions k % stride == offset are
    checked.  Returns the number of images checked."""
    import numpy as np

    from heif_amd.synthetic import permutation
    from oracle import oracle

    tiles, (ho, hl) = oracle.list_tiles(src)
    hvcc = src[ho:ho + hl]
    tw, th = info.tile_width, info.tile_height
    with cf.ThreadPoolExecutor(max(1, threads)) as ex:  # ctypes releases the GIL
        ref = list(ex.map(lambda t: oracle.decode_tile(hvcc, src[t[0]:t[0] + t[1]], tw, th), tiles))
    n, cols = info.num_tiles, info.grid_cols
    for s, o in zip(seeds, outs):
        perm = permutation(n, s)
        planes = [t.cpu().numpy().astype(np.uint16) for t in (o.y, o.cb, o.cr) if t is not None]
        for k in range(offset, n, stride):
            r, c = divmod(k, cols)
            for ci, pl in enumerate(planes):
                sh = 1 if ci else 0
                w, h = tw >> sh, th >> sh
                win = pl[h * r:h * (r + 1), w * c:w * (c + 1)]
                if not np.array_equal(win, ref[perm[k]][ci][:win.shape[0], :win.shape[1]]):
                    raise SystemExit(f"image seed {s} tile {k} plane {ci}: GPU planes differ from the oracle")
    return len(outs)


def config4u_files(S, seeds):
    """The distinct-tile control images; BENCH_C4U_CACHE names an .npz that
    keeps them between runs on one box (generation takes ~0.5 s per image)."""
    import numpy as np

    cache = os.environ.get("BENCH_C4U_CACHE")
    if cache and os.path.exists(cache):
        with np.load(cache) as z:
            if list(z["seeds"]) == list(seeds):
                return [z[f"f{i}"].tobytes() for i in range(len(seeds))]
    files = [S.config4u_image(s, threads=effective_cpus()) for s in seeds]
    if cache:
        np.savez(cache, seeds=np.array(seeds), **{f"f{i}": np.frombuffer(f, np.uint8) for i, f in enumerate(files)})
    return files


def verify_distinct(outs, files, info, stride, offset, threads) -> int:
    """Every given image (each with tiles of its own) against the oracle's
    decode of each of its tiles, placed in grid order.  Returns the number of
    images checked."""
    import numpy as np

    from oracle import oracle

    tw, th, n, cols = info.tile_width, info.tile_height, info.num_tiles, info.grid_cols
    with cf.ThreadPoolExecutor(max(1, threads)) as ex:
        for f, o in zip(files, outs):
            tiles, (ho, hl) = oracle.list_tiles(f)
            hvcc = f[ho:ho + hl]
            ks = list(range(offset, n, stride))
            ref = list(ex.map(lambda k: oracle.decode_tile(hvcc, f[tiles[k][0]:tiles[k][0] + tiles[k][1]], tw, th), ks))
            planes = [t.cpu().numpy().astype(np.uint16) for t in (o.y, o.cb, o.cr) if t is not None]
            for k, rk in zip(ks, ref):
                r, c = divmod(k, cols)
                for ci, pl in enumerate(planes):
                    sh = 1 if ci else 0
                    w, h = tw >> sh, th >> sh
                    win = pl[h * r:h * (r + 1), w * c:w * (c + 1)]
                    if not np.array_equal(win, rk[ci][:win.shape[0], :win.shape[1]]):
                        raise SystemExit(f"distinct-tile image: tile {k} plane {ci}: GPU planes differ from the oracle")
    return len(outs)


def end_to_end(H, ctx, files, outs0, n_batches, threads, stream, info) -> dict:
    """Host parse + pinned upload + decode of n_batches batches of `files`
    (re-parsed every time), two device batches reloaded alternately so the
    host work and upload of batch i+1 overlap the decode of batch i."""
    import torch

    outs = [outs0, ctx.alloc_outputs(H.HeifImage.parse_many(files[:len(outs0)], threads=threads))]
    batches = [None, None]
    t_parse = t_prep = 0.0
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(n_batches):
        ta = time.perf_counter()
        imgs = H.HeifImage.parse_many(files, threads=threads)
        tb = time.perf_counter()
        batches[i % 2] = ctx.prepare(imgs, reuse=batches[i % 2], wait=False)
        tc = time.perf_counter()
        batches[i % 2].decode_async(outs[i % 2], stream.cuda_stream)
        t_parse += tb - ta
        t_prep += tc - tb
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    for b in batches:
        if b is not None:
            if any(b.status(stream.cuda_stream)):
                raise SystemExit("e2e: decode status")
            b.free()
    px = info.width * info.height * len(files) * n_batches
    return {
        "value": round(px / dt / 1e6, 2),
        "unit": "Mpixels/s",
        "batches": n_batches,
        "images_per_batch": len(files),
        "ms_per_batch": round(dt / n_batches * 1e3, 3),
        "host_parse_ms_per_batch": round(t_parse / n_batches * 1e3, 3),
        "prepare_ms_per_batch": round(t_prep / n_batches * 1e3, 3),
        "host_threads": threads,
        "what": "HEIC files in host memory -> heifgpu_image_parse_many (thread pool) -> heifgpu_batch_prepare_ex "
                "(flatten into pinned memory, async H2D) -> decode; two batches alternate so host work and "
                "upload overlap the previous decode; planes stay in HBM",
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # (the round-end driver's K / W; the timed region holds the pipeline's fill and
    # drain, about 40 ms at 128 images, so K moves ms_per_step: 68.4 at 10, 66.5 at 20)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=128, help="images per GPU")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--workload", choices=["config4", "config5", "config4u"], default="config4",
                    help="config4u: config-4 geometry with 48 distinct synthetic tiles per image (control)")
    ap.add_argument("--verify", type=int, default=-1,
                    help="images checked bit-exact against the oracle on rank 0 (-1 = every image)")
    ap.add_argument("--split", choices=["images", "tiles"], default="images",
                    help="images: each rank its own shard (weak); tiles: every rank the same images, "
                         "tiles k %% world == rank (strong)")
    ap.add_argument("--parse", choices=["auto", "lanes", "solo", "spread"], default="auto",
                    help="CABAC parse mode (auto: solo for small batches, lanes otherwise)")
    ap.add_argument("--ppw", type=int, default=0, help="lanes mode: pictures per wave (0 = adaptive)")
    ap.add_argument("--no-e2e", action="store_true", help="skip the host-parse + upload + decode leg")
    ap.add_argument("--e2e-batches", type=int, default=6)
    ap.add_argument("--dry-run", action="store_true",
                    help="no GPU: only the rank launch, rendezvous (gloo) and timing reduction")
    args = ap.parse_args()
    tiles_split = args.split == "tiles"

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # plain `python bench.py --gpus N`: one child process per GPU, started
        # before anything here initialises HIP (torchrun sets WORLD_SIZE itself)
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    rank, world, local = dist_env()
    if "WORLD_SIZE" in os.environ and world != args.gpus:
        print(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}; measuring {world} rank(s)",
              file=sys.stderr, flush=True)
    if args.dry_run:
        dry_run(args)
        return

    import torch

    # the CPU baseline's -march=native oracle must be selected before anything imports the oracle
    # (the CPU baseline runs on rank 0 at N=1 only)
    with_cpu = rank == 0 and world == 1 and not args.no_cpu_baseline
    cpu_build = native_oracle() if with_cpu else None
    if world > 1:
        import torch.distributed as dist

        dist.init_process_group("nccl" if torch.cuda.is_available() else "gloo")
    torch.cuda.set_device(local)

    import heif_amd as H
    from heif_amd.synthetic import permuted_heic

    c5 = args.workload == "config5"
    c4u = args.workload == "config4u"
    if c5:
        from heif_amd import synth_encoder as S
        from heif_amd.synthetic import permutation

        p5 = S.CONFIG5["params"]
        pool = [S.picture(p5, 5000 + k) for k in range(135)]
        src = S.grid_heic(S.CONFIG5["out_w"], S.CONFIG5["out_h"], p5, pictures=pool)
    else:
        src = SAMPLE.read_bytes()
    seeds = list(range(args.batch)) if tiles_split else shard_seeds(args.batch, rank)
    if c5:
        files = [S.grid_heic(S.CONFIG5["out_w"], S.CONFIG5["out_h"], p5,
                             pictures=[pool[j] for j in permutation(135, s)]) for s in seeds]
    elif c4u:
        from heif_amd import synth_encoder as S

        files = config4u_files(S, seeds)
        src = files[0]
    else:
        files = [permuted_heic(src, s) for s in seeds]
    # host demux + parameter sets + slice headers alone (heifgpu_image_parse_many)
    host_threads = effective_cpus()
    t0 = time.perf_counter()
    images = H.HeifImage.parse_many(files, threads=1)
    host_parse_ms = (time.perf_counter() - t0) * 1e3 / len(files)
    t0 = time.perf_counter()
    images = H.HeifImage.parse_many(files, threads=host_threads)
    host_parse_ms_mt = (time.perf_counter() - t0) * 1e3 / len(files)
    info = images[0].info
    ctx = H.DecodeContext(local)
    # a tile split's planes sit in one buffer: one IPC handle per rank for the gather to rank 0
    outs, outbuf = ctx.alloc_outputs_contiguous(images) if tiles_split else (ctx.alloc_outputs(images), None)
    stride, offset = (world, rank) if tiles_split else (1, 0)
    t0 = time.perf_counter()
    batch = ctx.prepare(images, tile_stride=stride, tile_offset=offset, parse=args.parse, pics_per_wave=args.ppw)
    upload_s = time.perf_counter() - t0
    stream = torch.cuda.Stream(device=local)

    def step():
        batch.decode_async(outs, stream.cuda_stream)

    for _ in range(args.warmup):
        step()
    st = batch.status(stream.cuda_stream)
    if any(st):
        raise SystemExit(f"rank {rank}: decode status {st}")

    def barrier():
        if world > 1:
            torch.distributed.barrier()

    # HIP events around every kernel on the stream it runs on (internal parse /
    # recon streams), recorded through the timed region: per-kernel means over
    # the K timed steps, overlap included
    ctx.set_timing(True)
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()  # asynchronous: the parse of step n+1 overlaps the reconstruction of step n
    torch.cuda.synchronize()
    barrier()
    elapsed = time.perf_counter() - t0
    per_step = ctx.stage_times()
    if world > 1:
        t = torch.tensor([elapsed], device=f"cuda:{local}")
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        elapsed = float(t.item())
    st = batch.status(stream.cuda_stream)
    if any(st):
        raise SystemExit(f"rank {rank}: decode status {st}")

    # one more decode after the timed region, alone: the single-decode latency,
    # wall clock from the call to the planes being ready (streaming mode
    # overlaps the stages, so their sum is not the latency)
    torch.cuda.synchronize()
    t_lat = time.perf_counter()
    step()
    stream.synchronize()
    latency_ms = (time.perf_counter() - t_lat) * 1e3
    alone = ctx.stage_times()
    ctx.set_timing(False)

    # Row e2 across processes (outside the timed region): the tile split's
    # planes gathered to rank 0 over IPC + xGMI (heif_amd/tile_split.py).  In
    # the image split (default), one image is decoded tile-split for this check.
    gather = None
    g_full, g_seeds = None, None
    if world > 1 and not c4u:  # (the distinct-tile control is a one-GPU measurement)
        from heif_amd.tile_split import DeviceBackend, gather_to_rank0

        if tiles_split:
            g_imgs, g_outs, g_buf, g_seeds = images, outs, outbuf, seeds
        else:
            g_seeds = [0]
            g_imgs = [H.HeifImage.parse(files[0] if rank == 0 else permuted_heic(src, 0) if not c5 else
                                        S.grid_heic(S.CONFIG5["out_w"], S.CONFIG5["out_h"], p5,
                                                    pictures=[pool[j] for j in permutation(135, 0)]))]
            gb = ctx.prepare(g_imgs, tile_stride=world, tile_offset=rank)
            g_outs, g_buf = ctx.alloc_outputs_contiguous(g_imgs)
            gb.decode_async(g_outs, stream.cuda_stream)
            if any(gb.status(stream.cuda_stream)):
                raise SystemExit(f"rank {rank}: tile-split decode status")
            gb.free()
        g_full = ctx.alloc_outputs(g_imgs) if rank == 0 else None
        torch.cuda.synchronize()
        barrier()
        t0 = time.perf_counter()
        gather_to_rank0(DeviceBackend(H, ctx, stream), torch.distributed, g_outs, g_buf, g_full, rank, world)
        g_ms = (time.perf_counter() - t0) * 1e3
        if rank == 0:
            g_bytes = sum(t.numel() * t.element_size() for o in g_full for t in (o.y, o.cb, o.cr) if t is not None)
            gather = {"images": len(g_full), "ranks": world, "ms": round(g_ms, 3),
                      "bytes": g_bytes * (world - 1) // world,
                      "what": "each rank's tile subset (k % world == rank) gathered into rank 0's planes: handles "
                              "exchanged with all_gather_object, peers mapped with heifgpu_ipc_open, one "
                              "k_gather_tiles launch per image and rank reading over xGMI (ms includes the exchange "
                              "and the closing barrier)"}

    # --split tiles: every rank's own parse time, and the floor no tile split can
    # go below: the heaviest tile's parse decoded alone (its WPP chain; tiles are
    # independent pictures, /root/reference/src/heic/decoder.rs:114-119, so the
    # split removes tiles from a rank but never shortens that chain)
    split_parse = None
    if tiles_split:
        mine = {"rank": rank, "tiles": len(range(offset, info.num_tiles, stride)), "parse_ms": round(per_step[0], 3),
                "parse_ms_alone": round(alone[0], 3)}
        split_parse = [mine]
        if world > 1:
            split_parse = [None] * world
            torch.distributed.all_gather_object(split_parse, mine)
        if rank == 0:
            heavy = max(range(info.num_tiles), key=lambda k: images[0].tile_params(k)["payload_bytes"])
            fb = ctx.prepare(images[:1], tile_stride=info.num_tiles, tile_offset=heavy)
            f_outs = ctx.alloc_outputs(images[:1])
            ctx.set_timing(True)
            lat = []
            for _ in range(3):
                torch.cuda.synchronize()
                t_f = time.perf_counter()
                fb.decode_async(f_outs, stream.cuda_stream)
                stream.synchronize()
                lat.append((time.perf_counter() - t_f) * 1e3)
            f_parse = ctx.stage_times()[0]
            ctx.set_timing(False)
            if any(fb.status(stream.cuda_stream)):
                raise SystemExit("chain floor: decode status")
            fb.free()
            split_parse = {"per_rank": split_parse, "chain_floor": {
                "tile": heavy, "payload_bytes": images[0].tile_params(heavy)["payload_bytes"],
                "parse_ms": round(f_parse, 3), "latency_ms": round(min(lat), 3),
                "what": "the image's heaviest tile (payload bytes) decoded alone, spread parse: its WPP chain, "
                        "below which no rank's parse can go however the tiles are split"}}

    e2e = None
    if rank == 0 and world == 1 and not args.no_e2e:
        e2e = end_to_end(H, ctx, files, outs, args.e2e_batches, host_threads, stream, info)

    if rank == 0:
        verified = 0
        if args.verify:
            n_check = len(files) if args.verify < 0 else min(args.verify, len(files))
            if c4u:  # every image has its own tiles: each decoded by the oracle
                verified = verify_distinct(outs[:n_check], files[:n_check], info, stride, offset, host_threads)
            elif tiles_split and g_full is not None:  # the gathered images, every tile
                verified = verify_images(g_full[:n_check], g_seeds[:n_check], src, info, 1, 0, host_threads)
            else:
                verified = verify_images(outs[:n_check], seeds[:n_check], src, info, stride, offset, host_threads)
            if gather is not None and not tiles_split:
                gather["verified"] = verify_images(g_full, g_seeds, src, info, 1, 0, host_threads)
            elif gather is not None:
                gather["verified"] = verified
        px = info.width * info.height
        total_images = args.batch if tiles_split else args.batch * world
        value = total_images * px * args.steps / elapsed / 1e6  # every step decodes the whole batch
        parse_ms = per_step[0]  # k_parse time of one launch (one launch per step)
        chunks = 1
        coded_px = info.grid_cols * info.tile_width * info.grid_rows * info.tile_height
        bps = info.bytes_per_sample
        algo_per_image = info.coded_bytes + coded_px * 3 // 2 * bps  # compressed + coded planes
        # algorithmic bytes of this rank's launch (its tile share in a split)
        launch_bytes = args.batch * algo_per_image * len(range(offset, info.num_tiles, stride)) // info.num_tiles
        achieved = launch_bytes / (parse_ms / 1e3) / 1e9
        geom = batch.parse_geometry()
        kname = {"solo": "k_parse_solo<false>", "spread": "k_parse_solo<true>"}.get(
            geom["mode"], "k_parse_lanes")
        # counter evidence of this round (profiles/<round>/, written by tools/pmc_*.sh on the same
        # command): HBM bytes per launch (FETCH_SIZE / WRITE_SIZE passes) and the parse's SQ counters
        traffic, issue = None, None
        # config 5 has its own counter files (suffix _config5); config4u and split runs have none
        sfx = "_config5" if c5 else ""
        same_cfg = lambda j: (j.get("batch", j.get("batch_images")) == args.batch and not tiles_split and not c4u
                              and j.get("parse_mode", "lanes") == geom["mode"])
        try:
            tj = json.loads((PROFILES / f"pmc_traffic{sfx}.json").read_text())
            if same_cfg(tj):
                traffic = tj.get("k_parse_hbm_bytes_per_launch")
        except (OSError, ValueError):
            pass
        pj = None
        try:
            pj = json.loads((PROFILES / f"parse_counters_{geom['mode']}{sfx}.json").read_text())
            if not same_cfg(pj):
                pj = None
        except (OSError, ValueError):
            pj = None
        # bins per image: the oracle's count for halfmoonbay (every permutation the same);
        # config 5's from its counter file (tools/pmc_parse.sh counts them with the oracle)
        bpi = BINS_PER_IMAGE if not c5 and not c4u else (pj or {}).get("bins_per_image")
        bins = args.batch * bpi if bpi and not tiles_split else None
        if bins:
            issue = {"bins_per_launch": bins, "bins_per_s": round(bins / (parse_ms / 1e3), 1)}
            try:
                if pj:
                    pl, pw = pj["per_launch"], pj.get("per_wave", {})
                    valu, salu = pl["SQ_INSTS_VALU"] / bins, pl["SQ_INSTS_SALU"] / bins
                    issue.update({
                        "wave_instr_per_bin": round((pl["SQ_INSTS_VALU"] + pl["SQ_INSTS_SALU"] + pl["SQ_INSTS_LDS"]
                                                     + pl["SQ_INSTS_BRANCH"] + pl.get("SQ_INSTS_VMEM", 0)) / bins, 3),
                        "valu_per_bin": round(valu, 3), "salu_per_bin": round(salu, 3),
                        # one wave alone issues a VALU op every 4 cycles and an SALU op every cycle
                        # (MI355X_MICROARCH.md); SQ_WAVE_CYCLES counts quad-cycles
                        "issue_floor_frac": round((4 * pw["SQ_INSTS_VALU"] + pw["SQ_INSTS_SALU"])
                                                  / (4 * pw["SQ_WAVE_CYCLES"]), 4),
                        "wait_frac": round(pl["SQ_WAIT_ANY"] / pl["SQ_WAVE_CYCLES"], 4),
                        "source": f"profiles/{ROUND}/parse_counters_{geom['mode']}{sfx}.json",
                    })
            except (ValueError, KeyError, ZeroDivisionError):
                pass
        line = {
            "metric": ("Mpixels/s decoded (bit-exact) on 7680x4320 Main-10 HEIC batch" if c5 else
                       "Mpixels/s decoded (bit-exact) on 4032x3024 HEIC batch"),
            "value": round(value, 2),
            "unit": "Mpixels/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "strong" if tiles_split else "weak",
            "vs_baseline": None,
            "dtype": "u16" if c5 else "u8",
            "data": ("synthetic: 135 generated 10-bit tiles (heif_amd/synth_encoder.py) permuted per image" if c5 else
                     "synthetic: 48 distinct generated 8-bit tiles per image, no tile repeated in the batch "
                     "(heif_amd/synth_encoder.py CONFIG4U)" if c4u else
                     "synthetic: halfmoonbay.heic tiles permuted per image (mt19937_64 Fisher-Yates)"),
            "config": {
                "workload": f"config5 shard: {args.batch} x 7680x4320 10-bit 4:2:0 intra HEIC grids per GPU "
                            f"(135 tiles of 512x512, WPP)" if c5 else
                            f"config4 geometry, distinct tiles (control): {args.batch} x 4032x3024 8-bit 4:2:0 intra "
                            f"HEIC grid stills per GPU (48 tiles of 512x512, WPP)" if c4u else
                            f"config4 shard: {args.batch} x 4032x3024 8-bit 4:2:0 intra HEIC grid stills per GPU "
                            f"(48 tiles of 512x512, WPP)",
                "images_per_gpu": args.batch,
                "global_batch": total_images,
                "parallelism": (f"every image's grid tiles split k % {world} == rank over {world} GPU(s), "
                                "no collective on the data path" if tiles_split else
                                f"images sharded over {world} GPU(s), no collective on the data path"),
            },
            "roofline": {
                "bound": "hbm",
                "achieved": round(achieved, 2),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 6),
                "traffic": traffic,
                "traffic_source": f"profiles/{ROUND}/pmc_traffic{sfx}.json" if traffic else None,
                "kernel": kname,
                "parse_geometry": geom,
                "kernel_ms_per_launch": round(parse_ms / chunks, 3),
                "algorithmic_bytes_per_launch": launch_bytes // chunks,
                "launches_per_step": chunks,
                "binding": "per-bin CABAC dependency chain (issue / latency), not HBM: see `issue`",
                "issue": issue,
            },
            "stage_ms_per_step": {k: round(v, 3) for k, v in zip(
                ["parse", "transform", "intra", "deblock", "sao_out", "rbsp"], per_step)},
            "stage_ms_alone": {k: round(v, 3) for k, v in zip(
                ["parse", "transform", "intra", "deblock", "sao_out", "rbsp"], alone)},
            "pipeline": "three parse-output sets: decode n+2's k_rbsp+k_parse (parse stream), decode n+1's k_transform "
                        "(transform stream) and decode n's intra/deblock/SAO (recon stream) overlap; "
                        "the timed region includes the pipeline fill and drain; stage_ms_per_step are means over the "
                        "timed steps (overlap included), stage_ms_alone one decode with nothing beside it",
            "latency_ms_one_step": round(latency_ms, 3),  # wall clock, one decode alone (host launch included)
            "stage_ms_alone_sum": round(sum(alone), 3),
            "pipeline_hbm_gbs": round(launch_bytes / (elapsed / args.steps) / 1e9, 2),
            "host_parse_ms_per_image": round(host_parse_ms, 3),
            "host_parse_ms_per_image_mt": {"threads": host_threads, "ms": round(host_parse_ms_mt, 4)},
            "upload_s": round(upload_s, 3),
            "verified_images": verified,
        }
        if e2e:
            line["e2e"] = e2e
        if gather:
            line["tile_split_gather"] = gather
        if split_parse:
            line["tile_split_parse"] = split_parse
        if with_cpu:
            build = cpu_build
            threads = effective_cpus()
            label = "synthetic 10-bit" if c5 else "synthetic distinct 8-bit" if c4u else "halfmoonbay"
            cb = cpu_baseline(src, args.cpu_seconds, threads, label)
            one = cpu_baseline(src, min(args.cpu_seconds, 4.0), 1, label)
            cb["value_1core"] = one["value"]
            cb["host_cpus"] = os.cpu_count()
            cb["build"] = build
            cb["note"] = (f"one thread per CPU this job may use ({threads}: affinity and cgroup cpu.max); "
                          f"tiles are independent, so {os.cpu_count()} cores would scale to about "
                          f"{round(one['value'] * os.cpu_count())} Mpixels/s (1-core rate x cores, a projection, "
                          "not measured)")
            line["cpu_baseline"] = cb
        print(json.dumps(line), flush=True)
    batch.free()
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
