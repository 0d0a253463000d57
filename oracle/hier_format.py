"""numpy restatement of the gaussianhierarchy file formats, static traversal and Morton codes.

TEST INFRASTRUCTURE ONLY (imported by tests/, never by the product path).  The reference's loader/writer
(submodules/gaussianhierarchy/hierarchy_loader.cpp, hierarchy_writer.cpp) need Eigen, which is not vendored
(dependencies/eigen is empty), so they cannot be built here; the reference ships no .hier/.dhier files either.
Parity is therefore pinned on the byte layouts those files define, restated here field by field:

  .hier full    hierarchy_writer.cpp:43-56 / hierarchy_loader.cpp:39-65
  .hier half    hierarchy_writer.cpp:58-110 / hierarchy_loader.cpp:66-127 (binary16, round to nearest even:
                half.hpp:374, :820-835 -- numpy's float16 conversion rounds the same way)
  .dhier        hierarchy_writer.cpp:113-155 / hierarchy_loader.cpp:129-189 (node count forced to G, :185)
  traversal     traversal.cpp:15-39 (recExpand), recursive as written
  morton        morton.cu:9-42 (float32 arithmetic, truncating int64 conversion, 21 bits per axis)
"""
import numpy as np

SH_SIZE = [1, 4, 9, 16]


def write_dhier(path, pos, shs, opac, log_scales, rot, nodes, sh_degree, n_header=None):
    G = pos.shape[0]
    with open(path, "wb") as f:
        f.write(np.int32(G).tobytes())
        f.write(np.int32(sh_degree).tobytes())
        for a in (pos, rot, log_scales, opac):
            f.write(np.ascontiguousarray(a, np.float32).tobytes())
        f.write(np.ascontiguousarray(shs, np.float32).reshape(G, -1)[:, :3 * SH_SIZE[sh_degree]].tobytes())
        f.write(np.int32(nodes.shape[0] if n_header is None else n_header).tobytes())
        f.write(np.ascontiguousarray(nodes, np.int32).tobytes())


def read_dhier(path):
    b = open(path, "rb").read()
    G, deg = np.frombuffer(b, np.int32, 2)
    o = 8
    out = {}
    for k, w in (("pos", 3), ("rot", 4), ("log_scales", 3), ("opac", 1), ("shs", 3 * SH_SIZE[deg])):
        out[k] = np.frombuffer(b, np.float32, G * w, o).reshape(G, w)
        o += 4 * G * w
    o += 4  # stored node count: ignored, the loader uses G
    out["nodes"] = np.frombuffer(b, np.int32, G * 6, o).reshape(G, 6)
    out["sh_degree"] = int(deg)
    return out


def write_hier(path, pos, shs, opac, log_scales, rot, nodes, boxes, compressed=True):
    P, N = pos.shape[0], nodes.shape[0]
    f32 = lambda a: np.ascontiguousarray(a, np.float32)  # noqa: E731
    with open(path, "wb") as f:
        if not compressed:
            f.write(np.int32(P).tobytes())
            for a in (pos, rot, log_scales, opac, shs):
                f.write(f32(a).tobytes())
            f.write(np.int32(N).tobytes())
            f.write(np.ascontiguousarray(nodes, np.int32).tobytes())
            f.write(f32(boxes).tobytes())
            return
        f.write(np.int32(-P).tobytes())
        f.write(f32(pos).tobytes())
        for a in (rot, log_scales, opac, shs):
            f.write(f32(a).astype(np.float16).tobytes())
        f.write(np.int32(N).tobytes())
        nd = np.ascontiguousarray(nodes, np.int32)
        for i in range(N):  # HalfNode {parent, start, start_children; depth, count_children, count_leafs, count_merged}
            f.write(np.array([nd[i, 1], nd[i, 2], nd[i, 5]], np.int32).tobytes())
            f.write(np.array([nd[i, 0], nd[i, 6], nd[i, 3], nd[i, 4]], np.int16).tobytes())
        f.write(f32(boxes).astype(np.float16).tobytes())


def read_hier(path):
    b = open(path, "rb").read()
    P = int(np.frombuffer(b, np.int32, 1)[0])
    half = P < 0
    P = abs(P)
    o = 4
    out = {"pos": np.frombuffer(b, np.float32, P * 3, o).reshape(P, 3)}
    o += 12 * P
    dt, sz = (np.float16, 2) if half else (np.float32, 4)
    for k, w in (("rot", 4), ("log_scales", 3), ("opac", 1), ("shs", 48)):
        out[k] = np.frombuffer(b, dt, P * w, o).reshape(P, w).astype(np.float32)
        o += sz * P * w
    N = int(np.frombuffer(b, np.int32, 1, o)[0])
    o += 4
    if half:
        nodes = np.zeros((N, 7), np.int32)
        for i in range(N):
            pss = np.frombuffer(b, np.int32, 3, o)
            dccc = np.frombuffer(b, np.int16, 4, o + 12)
            o += 20
            nodes[i] = [dccc[0], pss[0], pss[1], dccc[2], dccc[3], pss[2], dccc[1]]
        out["boxes"] = np.frombuffer(b, np.float16, N * 8, o).reshape(N, 8).astype(np.float32)
    else:
        nodes = np.frombuffer(b, np.int32, N * 7, o).reshape(N, 7)
        o += 28 * N
        out["boxes"] = np.frombuffer(b, np.float32, N * 8, o).reshape(N, 8)
    out["nodes"] = nodes
    out["half"] = half
    return out


def expand_to_target(nodes, target):
    """traversal.cpp:15-39, recursive as written."""
    out = []

    def rec(i):
        depth, _parent, start, leafs, merged, start_children, n_children = (int(v) for v in nodes[i])
        out.extend(range(start, start + leafs))
        if depth <= target:
            out.extend(range(start + leafs, start + leafs + merged))
        else:
            for c in range(n_children):
                rec(start_children + c)

    rec(0)
    return np.array(out, np.int32)


def morton_codes(xyz, mn, mx):
    """morton.cu:9-42 in float32."""
    xyz, mn, mx = (np.asarray(a, np.float32) for a in (xyz, mn, mx))
    box = (mx - mn).astype(np.float32)
    p = ((xyz - mn) / box).astype(np.float32) * np.float32(1 << 21)
    q = p.astype(np.int64)
    code = np.zeros(len(xyz), np.int64)
    for i in range(21):
        for a in range(3):
            code |= ((q[:, a] >> i) & 1) << (3 * i + a)
    return code
