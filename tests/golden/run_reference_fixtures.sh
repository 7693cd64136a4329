#!/bin/bash
# Regenerate tests/golden/*.npz from the reference (this container only).
set -euo pipefail
HERE=$(cd "$(dirname "$0")" && pwd)
REF=$("$HERE/../../oracle/pyref/setup_ref.sh")
cd /tmp
env -u PYTHONPATH PYTHONPATH="$REF/shims:$REF" TORCH_EXTENSIONS_DIR="$REF/torch_ext" \
    python "$HERE/gen_reference_fixtures.py" "$@"
