"""Host AddressSanitizer + UBSan run over the host C++ that parses untrusted bytes (SURVEY.md
section 5, "Race detection / sanitizers"): the JPEG header parser and the decoder's per-thread
functions over a corrupt-JPEG corpus, the encoder's block functions on odd sizes, and the
composite plan on adversarial shifts.  CPU only (tools/host_sanitize.sh)."""
from __future__ import annotations

import os
import subprocess

from conftest import ROOT


def test_host_sanitizers_clean(tmp_path):
    r = subprocess.run(["bash", os.path.join(ROOT, "tools", "host_sanitize.sh"), str(tmp_path / "san")],
                       capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-6000:])
    assert "sanitize ok" in r.stdout
    assert '"inconsistent": 0' in r.stdout
