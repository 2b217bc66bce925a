"""Mutation fuzzing of the host parse + the kernels compiled for the host
under ASan/UBSan (heif_amd/csrc: `make emu`).  Seeds: halfmoonbay and
synthetic streams with tiles, slice segments, PCM + 4:4:4, a 4:2:2 grid and
scaling lists; each mutant flips / overwrites 1-8 bytes (for halfmoonbay in
its first 4 KB: the boxes and parameter sets).  A mutant fails when a
sanitizer reports or the harness exits with anything but 0 (parity), 1
(status bits / oracle disagreement) or 3 (host rejection); failing mutants
are kept under /tmp/fz.
usage: python tools/fuzz_emu.py N STAGES [ROUND]   (STAGES 0: host only, 5: every kernel)
HEIFGPU_PARSE=lanes|solo|spread picks the parse geometry.
"""
import concurrent.futures as cf
import os
import random
import subprocess
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import heif_amd.synth_encoder as S
exe = os.path.join(ROOT, 'heif_amd/csrc/build/emu/emu_check')
def P(**kw): return S.SynthParams(**{**dict(width=128, height=96), **kw})
seeds = {
  'hmb': open(os.path.join(ROOT, 'tests/golden/halfmoonbay.heic'), 'rb').read(),
  'tiles': S.single_heic(P(tile_cols=2, tile_rows=2, wpp=0), seed=1),
  'slices': S.single_heic(P(slice_ctus=4, slice_dependent=2, wpp=1, height=192), seed=1),
  'pcm444': S.single_heic(P(chroma_format=3, pcm=1, pcm_pct=30), seed=1),
  'grid': S.grid_heic(300, 200, P(chroma_format=2), seed=1),
  'scal': S.single_heic(P(scaling_list=1, bit_depth=10), seed=1),
}
env = dict(os.environ, ASAN_OPTIONS='exitcode=99:detect_leaks=0', UBSAN_OPTIONS='halt_on_error=1:exitcode=98')
def run(args):
    name, i, stages = args
    rng = random.Random(i * 7919 + sum(name.encode()) + 100000 * int(sys.argv[3] if len(sys.argv) > 3 else 0))
    d = bytearray(seeds[name])
    # mutate the header-heavy part: the first 4 KB (boxes) and, for small files, anywhere
    span = min(len(d), 4096 if name == 'hmb' else len(d))
    for _ in range(rng.choice([1, 2, 4, 8])):
        k = rng.randrange(span)
        op = rng.random()
        if op < 0.6: d[k] = rng.randrange(256)
        elif op < 0.8: d[k] ^= 1 << rng.randrange(8)
        else: d[k] = rng.choice([0, 0xff, 0x7f, 0x80])
    os.makedirs('/tmp/fz', exist_ok=True)
    path = f'/tmp/fz/m_{name}_{i}.heic'
    open(path, 'wb').write(d)
    r = subprocess.run([exe, path, str(stages)], capture_output=True, text=True, timeout=300, env=env)
    out = r.stdout + r.stderr
    bad = 'AddressSanitizer' in out or 'runtime error' in out or r.returncode not in (0, 1, 3)
    if not bad: os.remove(path)
    return name, i, r.returncode, bad, out[-1500:] if bad else ''
N = int(sys.argv[1]); stages = int(sys.argv[2])
jobs = [(n, i, stages) for n in seeds for i in range(N)]
nbad = 0
with cf.ThreadPoolExecutor(8) as ex:
    for name, i, rc, bad, out in ex.map(run, jobs):
        if bad:
            nbad += 1
            if nbad <= 5: print('BAD', name, i, rc, out)
print('done', len(jobs), 'bad', nbad)
