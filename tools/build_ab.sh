# Rebuild the current A/B set: one variant library per patch under tools/variants/ (NAME.patch -> lib/variants/NAME.so),
# each the current product sources with that patch applied (tools/build_variant.py --patch).  Variants measured in
# earlier rounds are in git history (tools/variants/INDEX.md, built with --rev).
set -e
cd "$(dirname "$0")/.."
python3 hierarchical-lod-gaussians_amd/hlgs_core/build.py
for p in tools/variants/*.patch; do
    [ -e "$p" ] || continue
    python3 tools/build_variant.py "$(basename "$p" .patch)" --patch "$p"
done
