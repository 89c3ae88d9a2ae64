"""The zero-copy pack reader (FqBulkReader) against the line-by-line FqReader (the restatement of
the reference's FqReader, pinned by the e2e fixtures): identical records and error text on
hostile FASTQ text -- CR/LF/CRLF mixes, blank lines, '@' resync garbage, length mismatches,
unterminated last lines, phred64, gzip -- with read buffers of a few bytes so the reference's
buffer-boundary rule for a '\\n' after a terminator (src/fqreader.cpp:139-140) is hit constantly,
and with packs of a few records so bytes are carried between pack arenas."""
import gzip
import random

import pytest

from fqtool_amd import abi


@pytest.fixture(scope="module")
def host():
    return abi.load_host()


def records(host, path, bulk, buf, pack_n=3, phred64=0):
    return abi.take_string(host, host.fqh_debug_records(path.encode(), bulk, buf, pack_n, phred64))


def hostile_text(rng, n, heavy=True):
    nl = [b"\n", b"\r\n", b"\r", b"\n\n", b"\r\n\n"] if heavy else [b"\n", b"\r\n"]
    p_bad = 0.03 if heavy else 0.002
    out = []
    for i in range(n):
        L = rng.choice([0, 1, 5, 17, 40] if heavy else [1, 5, 17, 40, 150])
        seq = bytes(rng.choice(b"ACGTN") for _ in range(L))
        qual = bytes(rng.randint(59, 104) for _ in range(L))
        if rng.random() < p_bad:
            qual = qual[:-1] if L else b"I"  # length mismatch: the input ends there
        if rng.random() < 0.05:
            out.append(b"garbage line" + rng.choice(nl))
        if rng.random() < 0.05:
            out.append(rng.choice(nl))
        t = lambda: rng.choice(nl) if rng.random() < 0.3 else b"\n"
        out.append(b"@r%d extra" % i + t() + seq + t() + b"+" + t() + qual + t())
    text = b"".join(out)
    if rng.random() < 0.5:
        text = text.rstrip(b"\r\n")  # unterminated last line
    return text


@pytest.mark.parametrize("seed", range(12))
def test_bulk_reader_equals_line_reader(host, tmp_path, seed):
    rng = random.Random(seed)
    text = hostile_text(rng, 60 if seed < 6 else 400, heavy=seed < 6)
    path = tmp_path / ("in.fq.gz" if seed % 3 == 2 else "in.fq")
    if seed % 3 == 2:
        path.write_bytes(gzip.compress(text))
    else:
        path.write_bytes(text)
    for buf in (3, 4, 7, 16, 61, 1000, 1 << 20):
        want = records(host, str(path), 0, buf, phred64=seed % 2)
        for pack_n in (1, 3, 50, 1000):
            got = records(host, str(path), 1, buf, pack_n, phred64=seed % 2)
            assert got == want, (buf, pack_n)


def test_bulk_reader_exact_multiple_of_buffer(host, tmp_path):
    rec = b"@a\r\nACGT\r\n+\r\nIIII\r\n"  # 20 bytes: CRLF terminators land on every buffer offset
    path = tmp_path / "m.fq"
    path.write_bytes(rec * 50)
    for buf in (5, 10, 19, 20, 21, 40, 100, 1000):
        want = records(host, str(path), 0, buf)
        assert records(host, str(path), 1, buf, 7) == want, buf
    # with 1 MiB buffers every record parses
    assert records(host, str(path), 1, 1 << 20, 7).count("\n") == 50


def plain_with_hazards(rng, n_rec, hazards):
    """Mostly plain FASTQ (several MiB, so the fast path splits it into segments) with a few hostile
    spots: CRLF or CR records, blank lines, garbage lines, qualities starting with '@' or '+',
    an empty sequence, a length mismatch (the input's last record)."""
    out = []
    spots = set(rng.sample(range(n_rec), hazards))
    for i in range(n_rec):
        L = rng.choice([36, 100, 150, 151, 250])
        seq = bytes(rng.choice(b"ACGTN") for _ in range(L))
        qual = bytearray(rng.randint(59, 104) for _ in range(L))
        if rng.random() < 0.02:
            qual[0] = ord(rng.choice("@+"))  # record-start look-alikes for the segment guess
        nl = b"\n"
        if i in spots:
            kind = rng.randrange(6)
            if kind == 5 and i < n_rec * 9 // 10:
                kind = 0  # (the mismatch only near the end: reading stops there)
            if kind == 0:
                nl = b"\r\n"
            elif kind == 1:
                out.append(b"\n")
            elif kind == 2:
                out.append(b"garbage\n")
            elif kind == 3:
                nl = b"\r"
            elif kind == 4:
                seq, qual = b"", bytearray()
            else:
                out.append(b"@x\nACGT\n+\nIII\n")  # length mismatch: reading stops here
        out.append(b"@r%d extra" % i + nl + seq + nl + b"+" + nl + bytes(qual) + nl)
    return b"".join(out)


@pytest.mark.parametrize("seed", range(6))
def test_parallel_fast_path_equals_line_reader(host, tmp_path, seed):
    rng = random.Random(100 + seed)
    text = plain_with_hazards(rng, 30000 if seed < 4 else 45000, [0, 1, 3, 8, 20, 0][seed])
    if seed == 5:
        text = text.rstrip(b"\n")  # unterminated last line
    path = tmp_path / "big.fq"
    path.write_bytes(text)
    want = records(host, str(path), 0, 1 << 20, phred64=seed % 2)
    assert want.count("\n") > 1000
    for pack_n in (1500, 7000, 100000):
        got = records(host, str(path), 2, 1 << 20, pack_n, phred64=seed % 2)
        assert got == want, pack_n
