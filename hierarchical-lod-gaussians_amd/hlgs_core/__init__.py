"""hlgs_core: host-side support for the MI355X rasterizer (library loading, build, synthetic scenes,
view-data-parallel gradient exchange)."""
