"""Parameter draws of the device image pipeline (host side): crop boxes inside the image, seeded reproducibility,
ColorJitter op order and no-op filtering."""
from bigdl_amd.dataset.device_pipeline import (BRIGHTNESS, CONTRAST, HUE, SATURATION, DeviceImagePipeline, _noop)
from bigdl_amd.utils.random_generator import RNG


def test_random_params_in_bounds_and_reproducible():
    pipe = DeviceImagePipeline(224, 224)
    shapes = [(375, 500, 3), (224, 224, 3), (50, 800, 3), (33, 33, 3)] * 5
    RNG.setSeed(3)
    a = pipe.random_params(shapes, jitter=dict(brightnessProb=1.0, contrastProb=1.0, saturationProb=1.0, hueProb=1.0))
    RNG.setSeed(3)
    b = pipe.random_params(shapes, jitter=dict(brightnessProb=1.0, contrastProb=1.0, saturationProb=1.0, hueProb=1.0))
    assert a == b
    for (H, W, _), p in zip(shapes, a):
        assert 0 <= p.y0 and p.y0 + p.ch <= H and 0 <= p.x0 and p.x0 + p.cw <= W and p.ch > 0 and p.cw > 0
        codes = [c for c, _ in p.ops]
        assert codes[0] == BRIGHTNESS and sorted(codes) == [BRIGHTNESS, CONTRAST, SATURATION, HUE]
        assert codes in ([BRIGHTNESS, CONTRAST, SATURATION, HUE], [BRIGHTNESS, SATURATION, HUE, CONTRAST])


def test_noop_amounts_match_host_skips():
    assert _noop(BRIGHTNESS, 0.0) and _noop(HUE, 0.0) and _noop(CONTRAST, 1.0005)
    assert not _noop(CONTRAST, 1.01) and not _noop(SATURATION, 1.0)
