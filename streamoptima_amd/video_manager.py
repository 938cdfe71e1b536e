"""YUV file I/O of the reference (video_manager.py:4-241, Encoder.read_yuv :110-126): the
path main.py takes from a raw 4:2:0 file to the Y planes the encoder consumes
(main.py:46-49: Video_Manager -> upscale_yuv420_to_yuv444 -> convert_yuv444_to_rgb ->
extract_y_only).  Host I/O around the GPU path, in numpy.

Same class, constructor, attributes and methods.  Deliberate differences:
  * the 4:2:0 reader reshapes to the `frames` the caller asked for; the reference's
    constructor always reshapes to 21 frames (its raw_yuv420_to_frame_arr default, :26,
    :62) and so cannot read any other length;
  * the matplotlib viewers (view_frame*, :99-142) and add_noise (:219-227, marked "doesn't
    really work" upstream) are out of scope and raise.
"""
from __future__ import annotations

import numpy as np


class Video_Manager:

    def __init__(self, raw_f, h_pixels, w_pixels, frames, v_type):
        self.current_f = raw_f
        self.h_pixels = h_pixels
        self.w_pixels = w_pixels
        self.frames = frames
        self.v_yuv420 = False
        self.v_yuv444 = False
        self.v_rgb = False
        self.vid_frames_yuv420 = None
        self.vid_frames_yuv444 = None
        self.vid_frames_rgb = None
        if v_type == "yuv_420":
            self.v_yuv420 = True
            self.num_y_p_yuv420 = int(h_pixels * w_pixels)
            self.num_u_p_yuv420 = int(self.num_y_p_yuv420 / 4)
            self.num_v_p_yuv420 = self.num_u_p_yuv420
            self.frame_size_p = self.num_y_p_yuv420 + self.num_u_p_yuv420 + self.num_v_p_yuv420
            self.vid_frames_yuv420 = self.raw_yuv420_to_frame_arr(raw_f, h_pixels, w_pixels, frames)
        elif v_type == "yuv_444":
            self.num_y_p_yuv_444 = int(h_pixels * w_pixels)
            self.num_u_p_yuv_444 = self.num_y_p_yuv_444
            self.num_v_p_yuv_444 = self.num_u_p_yuv_444
            self.frame_size_p = self.num_y_p_yuv_444 + self.num_u_p_yuv_444 + self.num_v_p_yuv_444
            self.v_yuv444 = False   # as the reference (:32): a 4:4:4 input is not marked available
            self.vid_frames_yuv444 = self.raw_yuv444_to_frame_arr(raw_f, h_pixels, w_pixels, frames)
        elif v_type == "rgb":
            print("[ERROR] Cannot parse RGB video file!")

    def print_status(self):
        print("################################################")
        print("Video Manager status")
        print("################################################")
        print("\tCurrent Video File  : ", self.current_f)
        print("\tVideo Height (in px): ", self.h_pixels)
        print("\tVideo Width (in px) : ", self.w_pixels)
        print("\tVideo # frames      : ", self.frames)
        print("\tYUV 4:2:0 available : ", self.v_yuv420)
        print("\tYUV 4:4:4 available : ", self.v_yuv444)
        print("\tRGB available       : ", self.v_rgb)
        print("################################################")

    @staticmethod
    def raw_yuv420_to_frame_arr(raw_yuv, h_pixel, w_pixel, frames=21, v_file=True):
        """[frames, H*W*1.5] uint8: each row one frame's planar Y | U | V (video_manager.py:62-77)."""
        raw = np.fromfile(raw_yuv, dtype="uint8") if v_file else np.asarray(raw_yuv)
        frame_size_p = int(h_pixel * w_pixel * 1.5)
        if frames is None:
            frames = raw.shape[0] // frame_size_p
        return raw.reshape(frames, frame_size_p)

    @staticmethod
    def raw_yuv444_to_frame_arr(raw_yuv, h_pixel, w_pixel, frames=300, v_file=True):
        """[frames, 3, H, W] uint8 (video_manager.py:84-97)."""
        raw = np.fromfile(raw_yuv, dtype="uint8") if v_file else np.asarray(raw_yuv)
        if frames is None:
            frames = raw.shape[0] // (3 * h_pixel * w_pixel)
        return raw.reshape(frames, 3, h_pixel, w_pixel)

    def upscale_yuv420_to_yuv444(self, replace=True):
        """Chroma upsampled by pixel repetition (video_manager.py:144-177); returns the flat
        concatenation of every frame's Y, U, V planes like the reference's hstack chain."""
        if self.v_yuv420 is False:
            print("[ERROR] No YUV 4:2:0 file available to convert!")
            return None
        ny, nu = self.num_y_p_yuv420, self.num_u_p_yuv420
        h2, w2 = int(self.h_pixels / 2), int(self.w_pixels / 2)
        f = self.frames
        src = self.vid_frames_yuv420[:f]
        y = src[:, :ny]
        u = src[:, ny:ny + nu].reshape(f, h2, w2).repeat(2, 1).repeat(2, 2).reshape(f, -1)
        v = src[:, ny + nu:ny + 2 * nu].reshape(f, h2, w2).repeat(2, 1).repeat(2, 2).reshape(f, -1)
        converted = np.concatenate([y, u, v], axis=1).reshape(-1)
        if replace:
            self.v_yuv444 = True
            self.vid_frames_yuv444 = self.raw_yuv444_to_frame_arr(converted, self.h_pixels, self.w_pixels, self.frames,
                                                                  False)
            self.num_y_p_yuv_444 = self.num_y_p_yuv420
            self.num_u_p_yuv_444 = self.num_y_p_yuv_444
            self.num_v_p_yuv_444 = self.num_y_p_yuv_444
        return converted

    def convert_yuv444_to_rgb(self, replace=True):
        """BT.601 studio-swing YUV -> RGB in float32, clipped to uint8 (video_manager.py:179-216):
        [frames, H, W, 3]."""
        if self.v_yuv444 is False:
            print("[ERROR] No YUV 4:4:4 file available to convert!")
            return None
        conv_mat = np.array([[1.164, 0.000, 2.018], [1.164, -0.813, -0.391], [1.164, 1.596, 0.000]])
        yuv = np.moveaxis(self.vid_frames_yuv444[: self.frames], 1, -1).astype(np.float32)   # [f, H, W, 3]
        yuv[..., 0] = yuv[..., 0].clip(16, 235) - 16
        yuv[..., 1:] = yuv[..., 1:].clip(16, 240) - 128
        rgb = np.matmul(yuv, conv_mat.T).clip(0, 255).astype("uint8")
        if replace:
            self.v_rgb = True
            self.vid_frames_rgb = rgb
            self.num_r_p_rgb = self.num_y_p_yuv_444
            self.num_g_p_rgb = self.num_u_p_yuv_444
            self.num_b_p_rgb = self.num_v_p_yuv_444
        return rgb

    def extract_y_only(self, dump=True):
        """The Y planes [frames, H, W] (video_manager.py:229-236): the encoder's input."""
        if self.v_yuv444 is False:
            print("[ERROR] No YUV 4:4:4 file avialable. Currenlty, tool can only extract Y-Only files from YUV 4:4:4.")
            return None
        return self.vid_frames_yuv444[:, 0, :, :]

    def save_y_only(self, filename, y_data_list):
        with open(filename, "wb") as f:
            for data in y_data_list:
                f.write(np.asarray(data).tobytes())

    def _out_of_scope(self, *a, **k):
        raise NotImplementedError("matplotlib viewers / add_noise are out of scope (SURVEY.md §2 rows 17, 19)")

    view_frame_yuv420 = view_frame_yuv444 = view_frame_rgb = view_frame = add_noise = _out_of_scope
