"""An OpenEXR PIZ encoder written from the published format (OpenEXR's
ImfPizCompressor / ImfWav / ImfHuf algorithms), independently of the decoder
in my-mitsuba_amd/host/exr.cpp: TEST INFRASTRUCTURE for tests/test_exr_piz.py.

  piz_compress(chunk, channels, width, lines) -> bytes

`chunk` is the uncompressed scanline block as the file stores it (per line,
per channel sorted by name, `width` little-endian values); `channels` lists
the pixel types (1 HALF, 2 FLOAT) in that order.  The steps:
  1. split the block into 16-bit words, channel-major (all lines of channel
     0, then channel 1, ...), a FLOAT as two words;
  2. bitmap of the words used (zero implied), forward LUT onto 0..k-1;
  3. per channel and per 16-bit half of its values, the 2-D Haar-like
     wavelet wav2Encode (14-bit arithmetic when every word < 2^14);
  4. Huffman: frequencies, code lengths from a min-heap merge with an extra
     run-length pseudo-symbol, canonical codes, the length table packed with
     zero runs, then the codes with runs of equal words as (code, rlc, count).
The heap follows libstdc++'s make_heap / pop_heap / push_heap step by step,
so the code lengths (and with them the bytes) are the ones OpenEXR's own
hufBuildEncTable produces when built with that library."""
import struct

import numpy as np

HUF_ENCBITS = 16
HUF_ENCSIZE = (1 << HUF_ENCBITS) + 1
SHORT_ZEROCODE_RUN = 59
LONG_ZEROCODE_RUN = 63
SHORTEST_LONG_RUN = 2 + LONG_ZEROCODE_RUN - SHORT_ZEROCODE_RUN
LONGEST_LONG_RUN = 255 + SHORTEST_LONG_RUN


# ---- libstdc++ heap algorithms (bits/stl_heap.h), comparator on values ----
def _push_heap(h, hole, top, value, comp):
    parent = (hole - 1) // 2
    while hole > top and comp(h[parent], value):
        h[hole] = h[parent]
        hole = parent
        parent = (hole - 1) // 2
    h[hole] = value


def _adjust_heap(h, hole, length, value, comp):
    top = hole
    second = hole
    while second < (length - 1) // 2:
        second = 2 * (second + 1)
        if comp(h[second], h[second - 1]):
            second -= 1
        h[hole] = h[second]
        hole = second
    if (length & 1) == 0 and second == (length - 2) // 2:
        second = 2 * (second + 1)
        h[hole] = h[second - 1]
        hole = second - 1
    _push_heap(h, hole, top, value, comp)


def make_heap(h, n, comp):
    if n < 2:
        return
    parent = (n - 2) // 2
    while True:
        _adjust_heap(h, parent, n, h[parent], comp)
        if parent == 0:
            return
        parent -= 1


def pop_heap(h, n, comp):
    if n > 1:
        last = n - 1
        value = h[last]
        h[last] = h[0]
        _adjust_heap(h, 0, last, value, comp)


def push_heap(h, n, comp):
    _push_heap(h, n - 1, 0, h[n - 1], comp)


# ---- Huffman (ImfHuf.cpp) --------------------------------------------------
def huf_build_enc_table(freq):
    """Code lengths -> canonical (code << 6 | length) per symbol; returns
    (hcode, im, iM) where iM is the run-length pseudo-symbol."""
    frq = [int(f) for f in freq]
    im = 0
    while not frq[im]:
        im += 1
    hlink = list(range(HUF_ENCSIZE))
    heap = []
    iM = im
    for i in range(im, HUF_ENCSIZE):
        if frq[i]:
            heap.append(i)
            iM = i
    iM += 1
    frq[iM] = 1
    heap.append(iM)
    nf = len(heap)
    comp = lambda a, b: frq[a] > frq[b]   # FHeapCompare: min-heap on frq  # noqa: E731
    make_heap(heap, nf, comp)
    scode = [0] * HUF_ENCSIZE
    while nf > 1:
        mm = heap[0]
        pop_heap(heap, nf, comp)
        nf -= 1
        m = heap[0]
        pop_heap(heap, nf, comp)
        frq[m] += frq[mm]
        push_heap(heap, nf, comp)
        j = m
        while True:
            scode[j] += 1
            if hlink[j] == j:
                hlink[j] = mm
                break
            j = hlink[j]
        j = mm
        while True:
            scode[j] += 1
            if hlink[j] == j:
                break
            j = hlink[j]
    # hufCanonicalCodeTable
    n = [0] * 59
    for l in scode:
        n[l] += 1
    c = 0
    for i in range(58, 0, -1):
        nc = (c + n[i]) >> 1
        n[i] = c
        c = nc
    hcode = [0] * HUF_ENCSIZE
    for i, l in enumerate(scode):
        if l > 0:
            hcode[i] = l | (n[l] << 6)
            n[l] += 1
    return hcode, im, iM


class BitWriter:
    def __init__(self):
        self.out = bytearray()
        self.c = 0
        self.lc = 0

    def bits(self, n, v):
        self.c = (self.c << n) | v
        self.lc += n
        while self.lc >= 8:
            self.lc -= 8
            self.out.append((self.c >> self.lc) & 0xFF)
        self.c &= (1 << self.lc) - 1 if self.lc else 0

    def code(self, hc):
        self.bits(hc & 63, hc >> 6)

    def flush(self):
        nbits = 8 * len(self.out) + self.lc
        if self.lc:
            self.out.append((self.c << (8 - self.lc)) & 0xFF)
        return bytes(self.out), nbits


def huf_pack_enc_table(hcode, im, iM):
    w = BitWriter()
    i = im
    while i <= iM:
        l = hcode[i] & 63
        if l == 0:
            zerun = 1
            while i < iM and zerun < LONGEST_LONG_RUN:
                if hcode[i + 1] & 63:
                    break
                i += 1
                zerun += 1
            if zerun >= 2:
                if zerun >= SHORTEST_LONG_RUN:
                    w.bits(6, LONG_ZEROCODE_RUN)
                    w.bits(8, zerun - SHORTEST_LONG_RUN)
                else:
                    w.bits(6, SHORT_ZEROCODE_RUN + zerun - 2)
                i += 1
                continue
        w.bits(6, l)
        i += 1
    return w.flush()[0]


def huf_compress(raw, rlmin=None):
    """rlmin: None -> a run is sent as (code, rlc, count) when that is shorter
    than repeating the code (current OpenEXR sendCode); an integer -> when
    the run is longer than rlmin (the fixed threshold of older releases)."""
    raw = [int(v) for v in raw]
    if not raw:
        return b""
    freq = np.bincount(np.asarray(raw, np.int64), minlength=HUF_ENCSIZE)
    hcode, im, iM = huf_build_enc_table(freq)
    table = huf_pack_enc_table(hcode, im, iM)
    w = BitWriter()
    rlc = hcode[iM]

    def send(s, cs):
        sc = hcode[s]
        if (cs > rlmin) if rlmin is not None else ((sc & 63) + (rlc & 63) + 8 < (sc & 63) * cs):
            w.code(sc)
            w.code(rlc)
            w.bits(8, cs)
        else:
            for _ in range(cs + 1):
                w.code(sc)

    s, cs = raw[0], 0
    for v in raw[1:]:
        if v == s and cs < 255:
            cs += 1
        else:
            send(s, cs)
            cs = 0
        s = v
    send(s, cs)
    data, nbits = w.flush()
    return struct.pack("<IIIII", im, iM, len(table), nbits, 0) + table + data


# ---- wavelet (ImfWav.cpp) ---------------------------------------------------
def _wenc14(a, b):
    as_ = a - 65536 if a >= 32768 else a
    bs = b - 65536 if b >= 32768 else b
    ms = (as_ + bs) >> 1
    ds = as_ - bs
    return ms & 0xFFFF, ds & 0xFFFF


def _wenc16(a, b):
    ao = (a + (1 << 15)) & 0xFFFF
    m = (ao + b) >> 1
    d = ao - b
    if d < 0:
        m = (m + (1 << 15)) & 0xFFFF
    return m, d & 0xFFFF


def wav2_encode(buf, base, nx, ox, ny, oy, mx):
    w14 = mx < (1 << 14)
    enc = _wenc14 if w14 else _wenc16
    n = min(nx, ny)
    p, p2 = 1, 2
    while p2 <= n:
        oy1, oy2, ox1, ox2 = oy * p, oy * p2, ox * p, ox * p2
        py = base
        ey = base + oy * (ny - p2)
        while py <= ey:
            px = py
            ex = py + ox * (nx - p2)
            while px <= ex:
                p01, p10 = px + ox1, px + oy1
                p11 = p10 + ox1
                i00, i01 = enc(buf[px], buf[p01])
                i10, i11 = enc(buf[p10], buf[p11])
                buf[px], buf[p10] = enc(i00, i10)
                buf[p01], buf[p11] = enc(i01, i11)
                px += ox2
            if nx & p:
                p10 = px + oy1
                buf[px], buf[p10] = enc(buf[px], buf[p10])
            py += oy2
        if ny & p:
            px = py
            ex = py + ox * (nx - p2)
            while px <= ex:
                p01 = px + ox1
                buf[px], buf[p01] = enc(buf[px], buf[p01])
                px += ox2
        p, p2 = p2, p2 << 1


# ---- the PIZ block (ImfPizCompressor.cpp compress) ---------------------------
def piz_compress(chunk: bytes, channels, width: int, lines: int, rlmin=None) -> bytes:
    words = np.frombuffer(chunk, "<u2")
    per = [width * (1 if t == 1 else 2) for t in channels]          # words per line per channel
    line = sum(per)
    assert words.size == line * lines
    tmp = []
    starts = []
    for c, n in enumerate(per):
        off = sum(per[:c])
        starts.append(len(tmp))
        for y in range(lines):
            tmp.extend(int(v) for v in words[y * line + off:y * line + off + n])
    bitmap = np.zeros(8192, np.uint8)
    for v in set(tmp):
        bitmap[v >> 3] |= 1 << (v & 7)
    bitmap[0] &= 0xFE
    nz = np.flatnonzero(bitmap)
    mn, mxb = (int(nz[0]), int(nz[-1])) if nz.size else (8191, 0)
    lut = np.zeros(65536, np.int64)
    k = 0
    for i in range(65536):
        if i == 0 or (bitmap[i >> 3] >> (i & 7)) & 1:
            lut[i] = k
            k += 1
    max_value = k - 1
    tmp = [int(lut[v]) for v in tmp]
    for c, t in enumerate(channels):
        size = 1 if t == 1 else 2
        for j in range(size):
            wav2_encode(tmp, starts[c] + j, width, size, lines, width * size, max_value)
    out = struct.pack("<HH", mn, mxb)
    if mn <= mxb:
        out += bitmap[mn:mxb + 1].tobytes()
    huf = huf_compress(tmp, rlmin)
    return out + struct.pack("<i", len(huf)) + huf


def write_piz_exr(path, img, half=True):
    """A scanline OpenEXR file, B/G/R channels, PIZ (32 lines per chunk)."""
    h, w, _ = img.shape

    def attr(name, typ, data):
        return name.encode() + b"\0" + typ.encode() + b"\0" + struct.pack("<i", len(data)) + data
    ptype = 1 if half else 2
    chl = b"".join(c.encode() + b"\0" + struct.pack("<iB3xii", ptype, 0, 1, 1) for c in "BGR") + b"\0"
    hdr = (struct.pack("<II", 20000630, 2) + attr("channels", "chlist", chl) +
           attr("compression", "compression", bytes([4])) +
           attr("dataWindow", "box2i", struct.pack("<4i", 0, 0, w - 1, h - 1)) +
           attr("displayWindow", "box2i", struct.pack("<4i", 0, 0, w - 1, h - 1)) +
           attr("lineOrder", "lineOrder", b"\0") + attr("pixelAspectRatio", "float", struct.pack("<f", 1)) +
           attr("screenWindowCenter", "v2f", struct.pack("<2f", 0, 0)) +
           attr("screenWindowWidth", "float", struct.pack("<f", 1)) + b"\0")
    dt = "<f2" if half else "<f4"
    chunks = []
    for y0 in range(0, h, 32):
        ys = range(y0, min(h, y0 + 32))
        raw = b"".join(np.ascontiguousarray(img[y, :, c]).astype(dt).tobytes() for y in ys for c in (2, 1, 0))
        data = piz_compress(raw, [ptype] * 3, w, len(ys))
        if len(data) >= len(raw):
            data = raw
        chunks.append(struct.pack("<ii", y0, len(data)) + data)
    off = len(hdr) + 8 * len(chunks)
    table = b""
    for c in chunks:
        table += struct.pack("<Q", off)
        off += len(c)
    with open(path, "wb") as f:
        f.write(hdr + table + b"".join(chunks))


def read_exr_chunks(path):
    """(header fields, [(y, packed bytes)]) of a scanline EXR file."""
    d = open(path, "rb").read()
    p = 8
    info = {}
    while True:
        e = d.index(b"\0", p)
        name = d[p:e].decode()
        p = e + 1
        if not name:
            break
        e = d.index(b"\0", p)
        typ = d[p:e].decode()
        p = e + 1
        size = struct.unpack_from("<i", d, p)[0]
        p += 4
        v = d[p:p + size]
        p += size
        if name == "compression":
            info["compression"] = v[0]
        elif name == "dataWindow":
            info["dataWindow"] = struct.unpack("<4i", v)
        elif name == "channels":
            chans, q = [], 0
            while v[q]:
                e = v.index(b"\0", q)
                cname = v[q:e].decode()
                q = e + 1
                chans.append((cname, struct.unpack_from("<i", v, q)[0]))
                q += 16
            info["channels"] = chans
        info.setdefault("types", {})[name] = typ
    x0, y0, x1, y1 = info["dataWindow"]
    lpc = {0: 1, 1: 1, 2: 1, 3: 16, 4: 32}[info["compression"]]
    n = (y1 - y0 + lpc) // lpc
    offs = struct.unpack_from(f"<{n}Q", d, p)
    chunks = []
    for o in offs:
        y, size = struct.unpack_from("<ii", d, o)
        chunks.append((y, d[o + 8:o + 8 + size]))
    return info, chunks
