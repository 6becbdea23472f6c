"""PIZ decoding of OpenEXR files (host/exr.cpp, Bitmap::readOpenEXR's input
for EnvironmentMap, envmap.cpp:154-180) pinned by an independent encoder
(tests/piz_encoder.py, written from the published ImfPizCompressor / ImfWav
/ ImfHuf algorithms):

- the reference's own data/tests/envmap.exr (scenes/envmap.exr, PIZ, HALF
  B/G/R, 512x256): every chunk of the file re-encodes byte for byte from the
  image host/exr.cpp decodes.  The file was written by an OpenEXR release
  whose Huffman coder sends a run as (code, run code, count) only when it is
  longer than 32 (RLMIN); with that rule and libstdc++'s heap order the
  encoder reproduces all 8 chunks.  PIZ is lossless and the encoder is a
  function of the image, so a decode that differed in any texel would not
  re-encode to the file;
- round trips of random HALF and FLOAT images of ragged sizes (a partial
  last chunk, widths not a multiple of the wavelet's 2^k blocks) through
  the current run-length rule."""
import os

import numpy as np
import pytest

import mtsg
from conftest import SCENES
from piz_encoder import piz_compress, read_exr_chunks, write_piz_exr

EXR = os.path.join(SCENES, "envmap.exr")


def test_reference_envmap_reencodes_byte_for_byte():
    info, chunks = read_exr_chunks(EXR)
    assert info["compression"] == 4 and [t for _, t in info["channels"]] == [1, 1, 1]
    img = mtsg.read_image(EXR)
    h, w, _ = img.shape
    names = [c for c, _ in info["channels"]]
    order = sorted(range(len(names)), key=lambda i: names[i])
    col = {"R": 0, "G": 1, "B": 2}
    assert len(chunks) == 8
    for y, data in chunks:
        ys = range(y, min(h, y + 32))
        raw = b"".join(np.ascontiguousarray(img[yy, :, col[names[i]]]).astype("<f2").tobytes()
                       for yy in ys for i in order)
        assert piz_compress(raw, [1, 1, 1], w, len(ys), rlmin=32) == data, f"chunk at y={y}"


@pytest.mark.parametrize("shape", [(37, 53), (70, 33), (32, 64), (5, 9)])
@pytest.mark.parametrize("half", [True, False], ids=["half", "float"])
def test_piz_round_trip(tmp_path, shape, half):
    rng = np.random.default_rng(sum(shape) + half)
    h, w = shape
    img = rng.gamma(2.0, 1.0, size=(h, w, 3)).astype(np.float32)
    img[: h // 3] = img[0, 0]                        # flat rows: long runs for the run-length code
    if half:
        img = img.astype(np.float16).astype(np.float32)
    p = tmp_path / "t.exr"
    write_piz_exr(str(p), img, half)
    np.testing.assert_array_equal(mtsg.read_image(str(p)), img)
