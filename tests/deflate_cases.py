"""Inputs of the deflate tests (tests/test_deflate_host.py, tests/test_gpu_deflate.py): the edge cases
of a block encoder and the demux writers' FASTQ shapes (records routed per sample, as fr_dmx_route
leaves them: one destination's records in their input order)."""
import numpy as np

from frender_amd import synth

DEFLATE_BLOCK = 1 << 16  # frd::BLOCK (frender_amd/csrc/fr_deflate_core.h)


def routed_fastq(n: int, R: int, seed: int = 5, samples: int = 96) -> bytes:
    """n synthetic records grouped by their code (first-appearance order of the codes, records in
    input order within a code): the bytes of a demux window, destination-major."""
    sheet = synth.make_sheet(samples, 8, 8)
    lines = synth.generate_bytes(sheet, 0, n, R=R, seed=seed).split(b"\n")
    groups = {}
    for i in range(0, len(lines) - 1, 4):
        groups.setdefault(lines[i].rsplit(b":", 1)[-1], []).append(b"\n".join(lines[i:i + 4]) + b"\n")
    return b"".join(b"".join(v) for v in groups.values())


def edge_cases() -> dict:
    rng = np.random.default_rng(7)
    B = DEFLATE_BLOCK
    text = b"".join(b"line %d of some text with repeats\n" % (i % 977) for i in range(6000))
    return {
        "empty": b"",
        "one": b"A",
        "five": b"ACGTN",
        "zeros_300k": bytes(300_000),
        "run_ab": b"ab" * 100_000,
        "random_200k": rng.integers(0, 256, 200_000, dtype=np.uint8).tobytes(),
        "block_exact": rng.integers(65, 69, B, dtype=np.uint8).tobytes(),
        "block_plus_1": rng.integers(65, 69, B + 1, dtype=np.uint8).tobytes(),
        "three_blocks_text": (text * 2)[: 3 * B - 5],
        "random_then_zeros": rng.integers(0, 256, 70_000, dtype=np.uint8).tobytes() + bytes(70_000),
        "fastq_r150": routed_fastq(2000, 150),
    }
