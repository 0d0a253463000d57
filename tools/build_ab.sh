# Rebuild the round-5 A/B variants against the current in-tree objects (each differs from C = libhlgs.so in one file):
#   sub4bwd the blend backward over 4x4 sub-block lists per row    tools/variants/raster_bwd_sub4.hip
#   sub4fwd the forward blend over 4x4 sub-block lists per row     tools/variants/raster_fwd_sub4.hip
#   pre04   the round-4 preprocess (register-staged SH rows)       tools/variants/preprocess_r04.hip
#   gbwd04  the round-4 Gaussian backward (per-lane record loads)  tools/variants/gauss_bwd_r04.hip
set -e
cd "$(dirname "$0")/.."
python3 hierarchical-lod-gaussians_amd/hlgs_core/build.py
python3 tools/build_variant.py sub4bwd tools/variants/raster_bwd_sub4.hip raster_bwd.hip
python3 tools/build_variant.py sub4fwd tools/variants/raster_fwd_sub4.hip raster_fwd.hip
python3 tools/build_variant.py pre04 tools/variants/preprocess_r04.hip preprocess.hip
python3 tools/build_variant.py gbwd04 tools/variants/gauss_bwd_r04.hip gauss_bwd.hip
