"""CPU oracle for the panorama hot path -- TEST INFRASTRUCTURE ONLY.

Nothing in ``vfx_image_stitching_amd`` imports this package.  Only ``tests/``,
``__graft_entry__.smoke()`` and the ``cpu_baseline`` leg of ``bench.py`` may use
it, and only as the checker / the timed CPU baseline, never as a product path.

Contents
--------
``cv2_compat``  restatement of the six OpenCV entry points the reference calls
                (cvtColor, resize, GaussianBlur, KeyPoint, imread, imwrite).
                The reference imports ``cv2`` at module top; OpenCV is absent
                here, so the golden-vector generator (tests/golden/make_golden.py)
                injects this module as ``sys.modules['cv2']``.
``sift``        vectorised numpy restatement of /root/reference/sift_impl.py.
``harris``      restatement of the Harris path of image_stitching_harris.py.
``stitch``      cylindrical projection, NN match, translation RANSAC, pad,
                blend, crop, drift and pano.txt parsing
                (image_stitching_sift.py / image_stitching_harris.py).

Pinning (see DESIGN.md "Oracle")
--------------------------------
* Harris path: pinned bit-exactly to the author's published panoramas
  (Result/harris_{prtn,grail}_result.jpg, pano_step_*/pano17.jpg) through
  SHA-256 digests committed in tests/golden/.
* Everything else: pinned to outputs of the reference's own Python, run in the
  build container against ``cv2_compat`` (tests/golden/make_golden.py).
  The SIFT path is "parity unpinned at the OpenCV boundary": real OpenCV
  accumulates GaussianBlur(f32) differently.
"""
