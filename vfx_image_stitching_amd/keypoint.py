"""cv2.KeyPoint-compatible record (cv2 is not assumed on the GPU box).

The reference creates keypoints with ``cv2.KeyPoint()`` / ``cv2.KeyPoint(x, y, size, angle,
response, octave)`` (sift_impl.py:206, 290) and reads ``pt``, ``size``, ``angle``,
``response``, ``octave``, ``class_id`` (sift_impl.py:299-358, sift_visualizeUI.py:64-75).
OpenCV stores the float fields as float32; reading them back yields Python floats of
those float32 values -- reproduced here so host-side arithmetic on keypoints (e.g. the
``dx = a[0] - b[0]`` of ransac) sees exactly the reference's numbers.
"""
from __future__ import annotations

import numpy as np

_f32 = np.float32


class KeyPoint:
    __slots__ = ("_x", "_y", "_size", "_angle", "_response", "octave", "class_id")

    def __init__(self, x=0.0, y=0.0, size=0.0, angle=-1.0, response=0.0, octave=0, class_id=-1):
        self._x = float(_f32(x))
        self._y = float(_f32(y))
        self._size = float(_f32(size))
        self._angle = float(_f32(angle))
        self._response = float(_f32(response))
        self.octave = int(octave)
        self.class_id = int(class_id)

    @property
    def pt(self):
        return (self._x, self._y)

    @pt.setter
    def pt(self, v):
        self._x = float(_f32(v[0]))
        self._y = float(_f32(v[1]))

    @property
    def size(self):
        return self._size

    @size.setter
    def size(self, v):
        self._size = float(_f32(v))

    @property
    def angle(self):
        return self._angle

    @angle.setter
    def angle(self, v):
        self._angle = float(_f32(v))

    @property
    def response(self):
        return self._response

    @response.setter
    def response(self, v):
        self._response = float(_f32(v))

    def __repr__(self):
        return (f"KeyPoint(pt={self.pt}, size={self.size}, angle={self.angle}, "
                f"response={self.response}, octave={self.octave})")


def from_records(rec: np.ndarray) -> list:
    """pano_kp records (structured array) -> list[KeyPoint]."""
    return [KeyPoint(float(r["x"]), float(r["y"]), float(r["size"]), float(r["angle"]),
                     float(r["response"]), int(r["octave"])) for r in rec]
