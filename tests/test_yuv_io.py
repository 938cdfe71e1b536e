"""YUV file I/O (video_manager.py:4-241, Encoder.read_yuv :110-126) against the reference's
own outputs on a 21-frame CIF 4:2:0 file (tests/golden/yuv_io.json, make_golden.py --only yuv),
and the top-level module names main.py imports (main.py:3-5)."""
import hashlib
import importlib
import json
import os

import numpy as np

from conftest import GOLDEN


def _sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def test_video_manager_and_read_yuv_match_reference(tmp_path):
    from streamoptima_amd.Encoder import Y_Video_codec
    from streamoptima_amd.synth import write_synth_yuv420
    from streamoptima_amd.video_manager import Video_Manager
    g = json.load(open(os.path.join(GOLDEN, "yuv_io.json")))
    path = str(tmp_path / "cif.yuv")
    write_synth_yuv420(path, g["frames"], g["h"], g["w"], seed=g["seed"])
    vm = Video_Manager(path, g["h"], g["w"], g["frames"], "yuv_420")
    assert list(vm.vid_frames_yuv420.shape) == g["yuv420_shape"] and _sha(vm.vid_frames_yuv420) == g["yuv420_sha"]
    up = vm.upscale_yuv420_to_yuv444()
    assert list(up.shape) == g["upscale_shape"] and _sha(up) == g["upscale_sha"]
    assert _sha(vm.vid_frames_yuv444) == g["yuv444_sha"]
    rgb = vm.convert_yuv444_to_rgb()
    assert list(rgb.shape) == g["rgb_shape"] and str(rgb.dtype) == g["rgb_dtype"] and _sha(rgb) == g["rgb_sha"]
    y = vm.extract_y_only()
    assert list(y.shape) == g["y_shape"] and _sha(y) == g["y_sha"]
    ry = Y_Video_codec.read_yuv(path, g["h"], g["w"], g["frames"])
    assert str(ry.dtype) == g["read_yuv_dtype"] and _sha(ry) == g["read_yuv_sha"]
    out = tmp_path / "y.yuv"
    vm.save_y_only(str(out), y)
    assert out.read_bytes() == np.ascontiguousarray(y).tobytes()


def test_video_manager_reads_other_lengths(tmp_path):
    """The reference can only read 21-frame files (its reshape default, video_manager.py:26,
    :62); here the requested frame count is used."""
    from streamoptima_amd.synth import synth_sequence, write_synth_yuv420
    from streamoptima_amd.video_manager import Video_Manager
    path = str(tmp_path / "s.yuv")
    write_synth_yuv420(path, 5, 64, 96, seed=3)
    vm = Video_Manager(path, 64, 96, 5, "yuv_420")
    vm.upscale_yuv420_to_yuv444()
    assert (vm.extract_y_only() == synth_sequence(5, 64, 96, 3)).all()


def test_top_level_modules_resolve():
    """main.py's `import video_manager`, `import Y_video_codec as codec`, `import decoder as
    dec` (main.py:3-5), and `import Encoder`, resolve to this package."""
    from streamoptima_amd.Encoder import Y_Video_codec
    from streamoptima_amd.decoder import decoder
    from streamoptima_amd.video_manager import Video_Manager
    assert importlib.import_module("Y_video_codec").Y_Video_codec is Y_Video_codec
    assert importlib.import_module("Encoder").Y_Video_codec is Y_Video_codec
    assert importlib.import_module("decoder").decoder is decoder
    assert importlib.import_module("video_manager").Video_Manager is Video_Manager
