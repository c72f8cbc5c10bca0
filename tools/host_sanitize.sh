#!/bin/bash
# Host AddressSanitizer + UndefinedBehaviorSanitizer run of the host C++ that parses untrusted
# input ("Race detection / sanitizers"; CPU only -- GPU sanitizers are not
# available on this pool):
#   * jpeg_host.cpp's header parser + frame planner and the decoder's per-thread functions
#     (jpeg_core.h, replayed on the host by tools/jpeg_sim.cpp) over a corrupt-JPEG corpus
#     (tools/make_fuzz_corpus.py: truncations, header bit flips, bad segment lengths, markers in
#     the scan, data after EOI);
#   * the encoder's per-block functions (tools/jpeg_enc_sim.cpp) on odd sizes;
#   * the composite plan (plan_core.h, tools/host_fuzz.cpp) on random and adversarial shifts.
# Any sanitizer report aborts with a non-zero status.  tests/test_sanitize.py runs this.
#
#   bash tools/host_sanitize.sh [OUT_DIR] [--small]
set -euo pipefail
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
OUT="${1:-/tmp/pano_sanitize}"
SMALL="${2:-}"
HIPCC="${HIPCC:-/opt/rocm/bin/hipcc}"
CSRC="$ROOT/vfx_image_stitching_amd/csrc"
mkdir -p "$OUT"
SAN=(-Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined
     -Xarch_host -fno-sanitize-recover=all -Xarch_host -fno-omit-frame-pointer)
CXX=("$HIPCC" --offload-arch=gfx950 -O1 -g -std=c++17 "${SAN[@]}")
"${CXX[@]}" -o "$OUT/jpeg_sim" "$ROOT/tools/jpeg_sim.cpp" "$CSRC/jpeg_host.cpp"
"${CXX[@]}" -o "$OUT/jpeg_enc_sim" "$ROOT/tools/jpeg_enc_sim.cpp" "$CSRC/jpeg_host.cpp"
"${CXX[@]}" -o "$OUT/host_fuzz" "$ROOT/tools/host_fuzz.cpp"
export ASAN_OPTIONS=detect_leaks=1:halt_on_error=1:abort_on_error=0
export UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1

rm -rf "$OUT/corpus"
NF=$(python3 "$ROOT/tools/make_fuzz_corpus.py" "$OUT/corpus" $SMALL)
find "$OUT/corpus" -name '*.jpg' -print0 | sort -z | xargs -0 -n 64 "$OUT/jpeg_sim" --batch > "$OUT/jpeg_sim.jsonl"
NL=$(wc -l < "$OUT/jpeg_sim.jsonl")
[ "$NL" -eq "$NF" ] || { echo "jpeg_sim: $NL status lines for $NF files"; exit 1; }
NOK=$(grep -c '"status": 0' "$OUT/jpeg_sim.jsonl" || true)
echo "jpeg decode: $NF corrupt/variant files, $NOK decoded, the rest refused with a status"

python3 - "$OUT" <<'EOF'
import sys, numpy as np
out = sys.argv[1]
rng = np.random.default_rng(3)
with open(f"{out}/enc_cases.txt", "w") as f:
    for h, w in ((1, 1), (1, 17), (9, 1), (7, 13), (16, 16), (17, 33), (64, 5), (100, 101)):
        p = f"{out}/enc_{h}x{w}.bgr"
        rng.integers(0, 256, (h, w, 3), dtype=np.uint8).tofile(p)
        f.write(f"{p} {h} {w}\n")
EOF
while read -r p h w; do
  for q in 1 50 95 100; do "$OUT/jpeg_enc_sim" "$p" "$h" "$w" "$q" "$OUT/enc.jpg"; done
done < "$OUT/enc_cases.txt"
echo "jpeg encode: clean"

"$OUT/host_fuzz" 20000 7
echo "sanitize ok"
