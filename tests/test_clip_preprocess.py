"""CLIP image preprocessing (src/embeddings/clip.py:129 -> HF CLIPImageProcessor).

Oracle: transformers' PIL-backed CLIPImageProcessor (the reference's processor; installed here, torchvision is
not, so it runs the PIL backend). The host CLIPProcessor must match it exactly (CPU test); the device kernel
(icap_clip_preprocess: Pillow's fixed-point two-pass bicubic resampler) must match it bit-for-bit on the
uint8 stage, i.e. to fp32 rounding of the normalisation (GPU test). Sizes cover down- and up-scaling, an axis
already at 224 (Pillow skips that pass) and odd aspect ratios.
"""

import warnings

import numpy as np
import pytest
import torch

SIZES = [(480, 640), (333, 500), (224, 300), (224, 224), (100, 1000), (517, 389), (1080, 1920), (225, 224)]


def _images(seed=0):
    from PIL import Image

    rng = np.random.default_rng(seed)
    out = []
    for h, w in SIZES:
        # smooth + noisy content so the resampler's rounding is exercised on both
        yy, xx = np.mgrid[0:h, 0:w]
        base = (127 + 100 * np.sin(xx / 17.0)[..., None] * np.cos(yy / 23.0)[..., None]).astype(np.int64)
        a = np.clip(base + rng.integers(-40, 41, (h, w, 3)), 0, 255).astype(np.uint8)
        out.append(Image.fromarray(a))
    return out


def _hf():
    warnings.filterwarnings("ignore")
    from transformers import CLIPImageProcessor

    return CLIPImageProcessor()


def test_host_processor_matches_hf():
    from icap.clip import CLIPProcessor

    hf, me = _hf(), CLIPProcessor()
    for im in _images():
        a = hf(images=im, return_tensors="np").pixel_values[0]
        b = me(im).pixel_values[0].numpy()
        assert np.array_equal(a, b), im.size


def test_geometry_matches_pillow_window():
    from icap import ops

    geo, _ = ops.clip_preprocess_geometry([(480, 640), (224, 300), (100, 1000)])
    # rows: src_off, in_h, in_w, new_h, new_w, top, left, tmp_off, y_first, tmp_rows
    # 480x640 -> 224x298, both axes resampled, the crop's vertical windows touch every source row
    assert geo[0][3:7] == [224, 298, 0, 37] and geo[0][8:] == [0, 480]
    # 224x300: the height is already 224, so Pillow skips the vertical pass: crop rows are source rows
    assert geo[1][3:5] == [224, 300] and geo[1][8:] == [0, 224]
    # 100x1000 upscaled to 224x2240 (scale < 1: unwidened kernel)
    assert geo[2][3:7] == [224, 2240, 0, 1008] and geo[2][8:] == [0, 100]


@pytest.mark.gpu
def test_device_preprocess_matches_hf(dev):
    from icap import ops

    hf = _hf()
    ims = _images(1)
    ref = np.stack([hf(images=im, return_tensors="np").pixel_values[0] for im in ims])
    got = ops.clip_preprocess([np.asarray(im) for im in ims], dev).cpu().numpy()
    assert got.shape == ref.shape
    assert np.abs(got - ref).max() <= 1e-6, [float(np.abs(got[i] - ref[i]).max()) for i in range(len(ims))]
