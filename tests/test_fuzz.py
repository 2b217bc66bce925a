"""Damaged streams of every coding layout the decoder takes: HEVC tiles,
slice segments (dependent, filtered across), PCM coding units, 4:2:2 and
4:4:4.  Each is corrupted three ways (random bytes, the second half zeroed,
the last eighth 0xff) and must end in status bits or a host rejection:
- on the CPU, the kernels compiled for the host under ASan/UBSan (`make emu`,
  halt on the first report) never read or write out of bounds;
- on the GPU, the corrupt images share one batch with a clean one, which
  stays bit-exact (no device fault, no cross-picture damage).

The reference's own robustness surface is its error returns
(src/hevc/rbsp_reader.rs, src/cabac/decoder.rs); this restates the same
contract for the decode the reference leaves todo!().
"""
import os
import pathlib
import random
import subprocess

import numpy as np
import pytest
from conftest import make_emu

S = pytest.importorskip("heif_amd.synth_encoder")

ROOT = pathlib.Path(__file__).resolve().parents[1]
CSRC = ROOT / "heif_amd" / "csrc"


def _p(**kw):
    return S.SynthParams(**{**dict(width=128, height=96), **kw})


BASES = {
    "pcm": _p(pcm=1, pcm_pct=40, width=256, height=192),
    "pcm422_10b": _p(chroma_format=2, bit_depth=10, pcm=1, pcm_pct=40, pcm_bd_c=7, wpp=0, width=256, height=192),
    "tiles444_across": _p(chroma_format=3, tile_cols=2, tile_rows=2, tile_lf_across=1, wpp=0, width=256, height=192),
    "slices_dep_across": _p(slice_ctus=4, slice_dependent=2, wpp=1, slice_lf_across=1, height=192),
    "tiles_nowpp": _p(tile_cols=3, tile_rows=2, wpp=0, width=256, height=192),
}
MODES = ("random", "zeroed", "tail")


def corrupt(name, mode):
    from oracle import oracle

    clean = S.single_heic(BASES[name], seed=3)
    items, _ = oracle.list_tiles(clean)
    d = bytearray(clean)
    rng = random.Random(7)
    for o, n in items:
        if mode == "random":
            for _ in range(40):
                d[o + 30 + rng.randrange(n - 30)] = rng.randrange(256)
        elif mode == "zeroed":
            d[o + n // 2:o + n] = bytes(n - n // 2)
        else:
            d[o + n - n // 8:o + n] = b"\xff" * (n // 8)
    return bytes(d)


@pytest.fixture(scope="module")
def emu_asan():
    make_emu("emu")
    return str(CSRC / "build" / "emu" / "emu_check")


@pytest.mark.parametrize("name", list(BASES))
def test_asan_kernels_survive_corrupt_layouts(emu_asan, tmp_path, name):
    env = dict(os.environ, ASAN_OPTIONS="exitcode=99:detect_leaks=0", UBSAN_OPTIONS="halt_on_error=1:exitcode=98")
    for mode in MODES:
        path = tmp_path / f"{name}_{mode}.heic"
        path.write_bytes(corrupt(name, mode))
        r = subprocess.run([emu_asan, str(path), "5"], capture_output=True, text=True, timeout=600, env=env)
        out = r.stdout + r.stderr
        assert "AddressSanitizer" not in out and "runtime error" not in out, (name, mode, out[-3000:])
        if r.returncode == 3:  # the host rejected the container / headers
            assert "host rejected" in out, out[-500:]
            continue
        assert r.returncode in (0, 1), (name, mode, out[-2000:])
        line = next(l for l in out.splitlines() if l.startswith("parse: status"))
        assert int(line.split()[2].rstrip(","), 16) != 0, (name, mode)


@pytest.mark.parametrize("parse", ["lanes", "spread", "solo"])
@pytest.mark.parametrize("mode", ["random", "zeroed"])
def test_asan_kernels_survive_corrupt_halfmoonbay(emu_asan, tmp_path, halfmoonbay, mode, parse):
    """The damaged halfmoonbay streams of test_emulation.py under ASan/UBSan
    (they once reached a QP outside 7.4.9.14's range and a scaling shift of 40)."""
    from test_emulation import _corrupt

    env = dict(os.environ, ASAN_OPTIONS="exitcode=99:detect_leaks=0", UBSAN_OPTIONS="halt_on_error=1:exitcode=98",
               HEIFGPU_PARSE=parse)
    path = tmp_path / f"{mode}.heic"
    path.write_bytes(_corrupt(halfmoonbay, mode))
    r = subprocess.run([emu_asan, str(path), "5"], capture_output=True, text=True, timeout=600, env=env)
    out = r.stdout + r.stderr
    assert "AddressSanitizer" not in out and "runtime error" not in out, out[-3000:]
    assert r.returncode in (0, 1), out[-2000:]
    line = next(l for l in out.splitlines() if l.startswith("parse: status"))
    assert int(line.split()[2].rstrip(","), 16) != 0


def _mutants(seed_name, data, n):
    """n deterministic mutants of `data`: 1-8 bytes overwritten / flipped anywhere
    (container boxes, parameter sets, slice headers or slice data)."""
    out = []
    for i in range(n):
        rng = random.Random(1000 * i + sum(seed_name.encode()))
        d = bytearray(data)
        for _ in range(rng.choice([1, 2, 4, 8])):
            k = rng.randrange(len(d))
            op = rng.random()
            if op < 0.6:
                d[k] = rng.randrange(256)
            elif op < 0.8:
                d[k] ^= 1 << rng.randrange(8)
            else:
                d[k] = rng.choice([0, 0xFF, 0x7F, 0x80])
        out.append(bytes(d))
    return out


@pytest.mark.parametrize("name", ["tiles_nowpp", "slices_dep_across", "pcm422_10b"])
def test_asan_mutation_fuzz(emu_asan, tmp_path, name):
    """Byte mutations of whole files (tools/fuzz_emu.py runs the long campaign):
    the host rejects, or the kernels end with status bits or parity, and no
    sanitizer reports anything.  The campaign found the ivlOffset, CuQpDeltaVal
    and terminate-bin cases the parse now clamps."""
    env = dict(os.environ, ASAN_OPTIONS="exitcode=99:detect_leaks=0", UBSAN_OPTIONS="halt_on_error=1:exitcode=98")
    for k, d in enumerate(_mutants(name, S.single_heic(BASES[name], seed=3), 12)):
        path = tmp_path / f"m{k}.heic"
        path.write_bytes(d)
        r = subprocess.run([emu_asan, str(path), "5"], capture_output=True, text=True, timeout=600, env=env)
        out = r.stdout + r.stderr
        assert "AddressSanitizer" not in out and "runtime error" not in out, (name, k, out[-3000:])
        assert r.returncode in (0, 1, 3), (name, k, r.returncode, out[-2000:])


# ------------------------------------------------------------------ GPU
torch = pytest.importorskip("torch")


@pytest.mark.gpu
@pytest.mark.parametrize("parse", ["lanes", "spread"])
def test_gpu_corrupt_layouts_set_status(oracle_mod, parse):
    """Every corrupt layout the host accepts, one batch per format with a clean
    image of that format: status bits on the damaged images, the clean one
    bit-exact."""
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import heif_amd as H

    ctx = H.DecodeContext(0)
    groups = {}
    for name, p in BASES.items():
        groups.setdefault((p.bit_depth, p.chroma_format), []).append(name)
    for (bd, cf), names in groups.items():
        clean = S.single_heic(BASES[names[0]], seed=11)
        datas, imgs = [], []
        for name in names:
            for mode in MODES:
                d = corrupt(name, mode)
                try:
                    im = H.HeifImage.parse(d)
                except H.HeifGpuError:
                    continue  # rejected by the host, like the emulation's "host rejected"
                datas.append(d)
                imgs.append(im)
        imgs.append(H.HeifImage.parse(clean))
        try:
            b = ctx.prepare(imgs, parse=parse)
        except H.HeifGpuError:
            # a batch-level rejection (e.g. a damaged slice layout): decode one by one
            b = None
        if b is None:
            kept = []
            for im in imgs[:-1]:
                try:
                    ctx.prepare([im], parse=parse).free()
                    kept.append(im)
                except H.HeifGpuError:
                    pass
            imgs = kept + [imgs[-1]]
            b = ctx.prepare(imgs, parse=parse)
        outs = ctx.alloc_outputs(imgs)
        b.decode_async(outs)
        st = b.status()
        assert all(s != 0 for s in st[:-1]) and st[-1] == 0, ((bd, cf), st)
        ref = oracle_mod.decode_heic(clean, with_checks=False)
        o = outs[-1]
        for g, r in zip((o.y, o.cb, o.cr), (ref.y, ref.cb, ref.cr)):
            assert np.array_equal(g.cpu().numpy().astype(np.uint16), r), (bd, cf)
        b.free()
    ctx.close()


@pytest.mark.gpu
@pytest.mark.parametrize("parse", ["lanes", "spread"])
def test_gpu_mutation_fuzz(oracle_mod, parse):
    """The mutants of test_asan_mutation_fuzz on the GPU, batched per format
    with a clean image: no device fault, status bits or clean output for the
    mutants, the clean image bit-exact."""
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import heif_amd as H

    ctx = H.DecodeContext(0)
    for name in ("tiles_nowpp", "slices_dep_across", "pcm422_10b"):
        clean = S.single_heic(BASES[name], seed=3)
        cimg = H.HeifImage.parse(clean)
        key = (cimg.info.bit_depth, cimg.info.chroma_format_idc)
        imgs = []
        for d in _mutants(name, clean, 12):
            try:
                im = H.HeifImage.parse(d)
                if (im.info.bit_depth, im.info.chroma_format_idc) != key:
                    continue
                ctx.prepare([im], parse=parse).free()  # the batch layout is accepted on its own
            except H.HeifGpuError:
                continue
            imgs.append(im)
        imgs.append(cimg)
        b = ctx.prepare(imgs, parse=parse)
        outs = ctx.alloc_outputs(imgs)
        b.decode_async(outs)
        st = b.status()
        assert st[-1] == 0, (name, st)
        ref = oracle_mod.decode_heic(clean, with_checks=False)
        o = outs[-1]
        for g, r in zip((o.y, o.cb, o.cr), (ref.y, ref.cb, ref.cr)):
            assert np.array_equal(g.cpu().numpy().astype(np.uint16), r), name
        b.free()
    ctx.close()
