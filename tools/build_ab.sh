# Rebuild the round-5 A/B variants against the current in-tree objects (each differs from C = libhlgs.so in one file):
#   r04bwd  the round-4 blend backward (8x8 quadrant passes)      tools/variants/raster_bwd_r04.hip
#   quadfwd the round-4 forward blend (one splat per iteration)    tools/variants/raster_fwd_quadpass.hip
#   pre04   the round-4 preprocess (register-staged SH rows)       tools/variants/preprocess_r04.hip
set -e
cd "$(dirname "$0")/.."
python3 hierarchical-lod-gaussians_amd/hlgs_core/build.py
python3 tools/build_variant.py r04bwd tools/variants/raster_bwd_r04.hip raster_bwd.hip
python3 tools/build_variant.py quadfwd tools/variants/raster_fwd_quadpass.hip raster_fwd.hip
python3 tools/build_variant.py pre04 tools/variants/preprocess_r04.hip preprocess.hip
#   gbwd04  the round-4 Gaussian backward (per-lane record loads)  tools/variants/gauss_bwd_r04.hip
python3 tools/build_variant.py gbwd04 tools/variants/gauss_bwd_r04.hip gauss_bwd.hip
