// hier_io.cpp -- host-side hierarchy file I/O and traversal of libhlgs.so (no Eigen, no torch).
//
// Byte formats (all little-endian, paths relative to submodules/gaussianhierarchy):
//   .hier, full   (hierarchy_writer.cpp:33-57 write(compressed=false), hierarchy_loader.cpp:39-65 load):
//       int32 P; P x float3 pos; P x float4 rot; P x float3 log-scale; P x float opacity; P x 48 float SH;
//       int32 N; N x Node (7 int32: depth, parent, start, count_leafs, count_merged, start_children,
//       count_children); N x Box (2 x float4: minn, maxx)
//   .hier, half   (write(compressed=true) :58-110 -- the default of WriteHierarchy; load :66-127):
//       int32 -P; P x float3 pos; then binary16 rot (4), log-scale (3), opacity (1), SH (48) per Gaussian,
//       each block contiguous; int32 N; N x HalfNode {int32 parent, start, start_children; int16 depth,
//       count_children, count_leafs, count_merged} (types.h:94-100); N x HalfBox (8 x binary16)
//   .dhier        (hierarchy_writer.cpp:113-155 writeDynamic, hierarchy_loader.cpp:129-189 loadDynamic):
//       int32 G; int32 sh_degree; G x float3 pos; G x float4 rot; G x float3 log-scale; G x float opacity;
//       G x 3 (deg+1)^2 float SH; int32 N (ignored by the loader: N = G); G x HierarchyNode (6 int32:
//       depth, parent, child_count, first_child, next_sibling, max_side_length)
// binary16 conversions round to nearest, ties to even (half.hpp HALF_ROUND_STYLE 1, half.hpp:820-835).
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <string>
#include <vector>

#include "../../include/hlgs.h"

namespace hlgs {
int fail_msg(int code, const std::string& msg);  // capi.hip

namespace {

// IEEE binary16 <-> binary32 (round to nearest even), bit-exact with half.hpp's default conversions.
uint16_t f2h(float f)
{
    uint32_t x;
    memcpy(&x, &f, 4);
    const uint32_t sign = (x >> 16) & 0x8000u;
    const uint32_t absx = x & 0x7fffffffu;
    if (absx >= 0x7f800000u) return (uint16_t)(sign | 0x7c00u | (absx > 0x7f800000u ? 0x200u | ((absx >> 13) & 0x3ffu) : 0u));
    if (absx >= 0x477ff000u) return (uint16_t)(sign | 0x7c00u);  // rounds to >= 65520: overflow to inf
    if (absx < 0x38800000u) {                                    // subnormal half (or zero)
        if (absx < 0x33000000u) return (uint16_t)sign;           // < 2^-25: rounds to 0
        const uint32_t e = absx >> 23, m = (absx & 0x7fffffu) | 0x800000u;
        const uint32_t shift = 126 - e;  // 14 + (113 - e) + ... so that result = m >> (shift)
        const uint32_t r = m >> shift, rem = m & ((1u << shift) - 1), half = 1u << (shift - 1);
        uint32_t h = r + ((rem > half || (rem == half && (r & 1u))) ? 1u : 0u);
        return (uint16_t)(sign | h);
    }
    const uint32_t e = (absx >> 23) - 112, m = absx & 0x7fffffu;
    uint32_t h = (e << 10) | (m >> 13);
    const uint32_t rem = m & 0x1fffu;
    if (rem > 0x1000u || (rem == 0x1000u && (h & 1u))) h++;
    return (uint16_t)(sign | h);
}

float h2f(uint16_t h)
{
    const uint32_t sign = (uint32_t)(h & 0x8000u) << 16;
    uint32_t e = (h >> 10) & 0x1fu, m = h & 0x3ffu, x;
    if (e == 0) {
        if (m == 0) x = sign;
        else {  // subnormal: normalise
            e = 113;
            while (!(m & 0x400u)) { m <<= 1; e--; }
            x = sign | (e << 23) | ((m & 0x3ffu) << 13);
        }
    } else if (e == 31) {
        x = sign | 0x7f800000u | (m << 13);
    } else {
        x = sign | ((e + 112) << 23) | (m << 13);
    }
    float f;
    memcpy(&f, &x, 4);
    return f;
}

struct File {
    FILE* f = nullptr;
    ~File() { if (f) fclose(f); }
};

bool rd(FILE* f, void* dst, size_t bytes) { return bytes == 0 || fread(dst, 1, bytes, f) == bytes; }
bool wr(FILE* f, const void* src, size_t bytes) { return bytes == 0 || fwrite(src, 1, bytes, f) == bytes; }

const int kShSize[4] = {1, 4, 9, 16};

}  // namespace
}  // namespace hlgs

using namespace hlgs;

extern "C" {

int hlgs_hier_info_read(const char* path, int dynamic, hlgs_hier_info* info)
{
    if (!path || !info) return fail_msg(HLGS_ERR_ARG, "null argument");
    memset(info, 0, sizeof(*info));
    File F;
    F.f = fopen(path, "rb");
    if (!F.f) return fail_msg(HLGS_ERR_ARG, "File not found!");
    // The header counts are checked against the file's size before anything is sized by them: the reference's loader
    // trusts them (hierarchy_loader.cpp:39-65, 129-189), which lets a malformed file drive huge or negative sizes.
    if (fseek(F.f, 0, SEEK_END) != 0) return fail_msg(HLGS_ERR_ARG, "unreadable hierarchy file");
    const long long fsize = (long long)ftell(F.f);
    if (fsize < 0 || fseek(F.f, 0, SEEK_SET) != 0) return fail_msg(HLGS_ERR_ARG, "unreadable hierarchy file");
    int32_t a = 0, b = 0;
    if (!rd(F.f, &a, 4)) return fail_msg(HLGS_ERR_ARG, "truncated hierarchy file");
    if (dynamic) {
        if (!rd(F.f, &b, 4)) return fail_msg(HLGS_ERR_ARG, "truncated hierarchy file");
        if (a < 0 || b < 0 || b > 3) return fail_msg(HLGS_ERR_ARG, "not a dynamic hierarchy (.dhier) file");
        const long long need = 8 + (long long)a * (12 + 16 + 12 + 4 + 12LL * kShSize[b]) + 4 + (long long)a * 24;
        if (need > fsize) return fail_msg(HLGS_ERR_ARG, "truncated hierarchy file");
        info->format = HLGS_HIER_DYNAMIC;
        info->G = a;
        info->sh_degree = b;
        info->N = a;  // hierarchy_loader.cpp:185: the node count is the Gaussian count
        return HLGS_OK;
    }
    const bool half = a < 0;
    const long long P = half ? -(long long)a : a;
    const long long per = half ? 12 + 2 * (4 + 3 + 1 + 48) : 12 + 16 + 12 + 4 + 4 * 48;
    if (4 + P * per + 4 > fsize || fseek(F.f, (long)(4 + P * per), SEEK_SET) != 0 || !rd(F.f, &b, 4))
        return fail_msg(HLGS_ERR_ARG, "truncated hierarchy file");
    if (b < 0) return fail_msg(HLGS_ERR_ARG, "negative node count in hierarchy file");
    const long long node_bytes = half ? 12 + 8 + 16 : 28 + 32;  // (Half)Node + (Half)Box
    if (4 + P * per + 4 + (long long)b * node_bytes > fsize) return fail_msg(HLGS_ERR_ARG, "truncated hierarchy file");
    info->format = half ? HLGS_HIER_HALF : HLGS_HIER_FULL;
    info->G = (int)P;
    info->N = b;
    info->sh_degree = 3;
    return HLGS_OK;
}

int hlgs_hier_load(const char* path, float* pos, float* rot, float* log_scales, float* opacities, float* shs, int* nodes,
                   float* boxes)
{
    hlgs_hier_info info;
    int rc = hlgs_hier_info_read(path, 0, &info);
    if (rc) return rc;
    File F;
    F.f = fopen(path, "rb");
    if (!F.f) return fail_msg(HLGS_ERR_ARG, "File not found!");
    const size_t P = (size_t)info.G, N = (size_t)info.N;
    int32_t hdr;
    bool ok = rd(F.f, &hdr, 4) && rd(F.f, pos, 12 * P);
    if (info.format == HLGS_HIER_FULL) {
        ok = ok && rd(F.f, rot, 16 * P) && rd(F.f, log_scales, 12 * P) && rd(F.f, opacities, 4 * P) &&
             rd(F.f, shs, 4 * 48 * P) && rd(F.f, &hdr, 4) && rd(F.f, nodes, 28 * N) && rd(F.f, boxes, 32 * N);
        if (!ok) return fail_msg(HLGS_ERR_ARG, "truncated hierarchy file");
        return HLGS_OK;
    }
    std::vector<uint16_t> h(P * 48 > N * 8 ? P * 48 : N * 8);
    auto block = [&](float* dst, size_t n) {
        if (!rd(F.f, h.data(), 2 * n)) return false;
        for (size_t i = 0; i < n; i++) dst[i] = h2f(h[i]);
        return true;
    };
    ok = ok && block(rot, 4 * P) && block(log_scales, 3 * P) && block(opacities, P) && block(shs, 48 * P);
    ok = ok && rd(F.f, &hdr, 4);
    if (!ok) return fail_msg(HLGS_ERR_ARG, "truncated hierarchy file");
    for (size_t i = 0; i < N; i++) {  // HalfNode -> Node (hierarchy_loader.cpp:111-119)
        int32_t pss[3];
        int16_t dccc[4];
        if (!rd(F.f, pss, 12) || !rd(F.f, dccc, 8)) return fail_msg(HLGS_ERR_ARG, "truncated hierarchy file");
        int* nd = nodes + 7 * i;
        nd[0] = dccc[0];  // depth
        nd[1] = pss[0];   // parent
        nd[2] = pss[1];   // start
        nd[3] = dccc[2];  // count_leafs
        nd[4] = dccc[3];  // count_merged
        nd[5] = pss[2];   // start_children
        nd[6] = dccc[1];  // count_children
    }
    if (!block(boxes, 8 * N)) return fail_msg(HLGS_ERR_ARG, "truncated hierarchy file");
    return HLGS_OK;
}

int hlgs_hier_write(const char* path, int G, int N, const float* pos, const float* shs, const float* opacities,
                    const float* log_scales, const float* rot, const int* nodes, const float* boxes, int compressed)
{
    if (!path || G < 0 || N < 0) return fail_msg(HLGS_ERR_ARG, "invalid argument");
    File F;
    F.f = fopen(path, "wb");
    if (!F.f) return fail_msg(HLGS_ERR_ARG, "File not created!");
    const size_t P = (size_t)G, NN = (size_t)N;
    if (!compressed) {
        bool ok = wr(F.f, &G, 4) && wr(F.f, pos, 12 * P) && wr(F.f, rot, 16 * P) && wr(F.f, log_scales, 12 * P) &&
                  wr(F.f, opacities, 4 * P) && wr(F.f, shs, 4 * 48 * P) && wr(F.f, &N, 4) && wr(F.f, nodes, 28 * NN) &&
                  wr(F.f, boxes, 32 * NN);
        return ok ? HLGS_OK : fail_msg(HLGS_ERR_ARG, "write failed");
    }
    for (size_t i = 0; i < NN; i++) {  // hierarchy_writer.cpp:90-92
        const int* nd = nodes + 7 * i;
        if (nd[0] > 32000 || nd[6] > 32000 || nd[3] > 32000 || nd[4] > 32000)
            return fail_msg(HLGS_ERR_ARG, "Would lose information!");
    }
    const int32_t indi = -G;
    std::vector<uint16_t> h(P * 48 > NN * 8 ? P * 48 : NN * 8);
    auto block = [&](const float* src, size_t n) {
        for (size_t i = 0; i < n; i++) h[i] = f2h(src[i]);
        return wr(F.f, h.data(), 2 * n);
    };
    bool ok = wr(F.f, &indi, 4) && wr(F.f, pos, 12 * P) && block(rot, 4 * P) && block(log_scales, 3 * P) &&
              block(opacities, P) && block(shs, 48 * P) && wr(F.f, &N, 4);
    for (size_t i = 0; ok && i < NN; i++) {
        const int* nd = nodes + 7 * i;
        const int32_t pss[3] = {nd[1], nd[2], nd[5]};
        const int16_t dccc[4] = {(int16_t)nd[0], (int16_t)nd[6], (int16_t)nd[3], (int16_t)nd[4]};
        ok = wr(F.f, pss, 12) && wr(F.f, dccc, 8);
    }
    ok = ok && block(boxes, 8 * NN);
    return ok ? HLGS_OK : fail_msg(HLGS_ERR_ARG, "write failed");
}

int hlgs_dhier_load(const char* path, float* pos, float* rot, float* log_scales, float* opacities, float* shs, int* nodes)
{
    hlgs_hier_info info;
    int rc = hlgs_hier_info_read(path, 1, &info);
    if (rc) return rc;
    File F;
    F.f = fopen(path, "rb");
    if (!F.f) return fail_msg(HLGS_ERR_ARG, "File not found!");
    const size_t G = (size_t)info.G;
    int32_t hdr[2], n_file;
    const bool ok = rd(F.f, hdr, 8) && rd(F.f, pos, 12 * G) && rd(F.f, rot, 16 * G) && rd(F.f, log_scales, 12 * G) &&
                    rd(F.f, opacities, 4 * G) && rd(F.f, shs, 12 * (size_t)kShSize[info.sh_degree] * G) &&
                    rd(F.f, &n_file, 4) && rd(F.f, nodes, 24 * G);
    return ok ? HLGS_OK : fail_msg(HLGS_ERR_ARG, "truncated hierarchy file");
}

int hlgs_dhier_write(const char* path, int G, int N, const float* pos, const float* shs, const float* opacities,
                     const float* log_scales, const float* rot, const int* nodes, int sh_degree)
{
    if (!path || G < 0 || N < 0 || sh_degree < 0 || sh_degree > 3) return fail_msg(HLGS_ERR_ARG, "invalid argument");
    File F;
    F.f = fopen(path, "wb");
    if (!F.f) return fail_msg(HLGS_ERR_ARG, "File not created!");
    const size_t P = (size_t)G;
    const bool ok = wr(F.f, &G, 4) && wr(F.f, &sh_degree, 4) && wr(F.f, pos, 12 * P) && wr(F.f, rot, 16 * P) &&
                    wr(F.f, log_scales, 12 * P) && wr(F.f, opacities, 4 * P) &&
                    wr(F.f, shs, 12 * (size_t)kShSize[sh_degree] * P) && wr(F.f, &N, 4) &&
                    wr(F.f, nodes, 24 * (size_t)N);
    return ok ? HLGS_OK : fail_msg(HLGS_ERR_ARG, "write failed");
}

// traversal.cpp:15-39 (recExpand from the root) as an explicit-stack pre-order walk: a node's leaf range, then --
// when its depth is <= target -- its merged range, otherwise its children in order.
int hlgs_expand_to_target(int N, const int* nodes, int target, int* out, int capacity, int* count)
{
    if (!nodes || !count || N < 0) return fail_msg(HLGS_ERR_ARG, "invalid argument");
    *count = 0;
    if (N == 0) return HLGS_OK;
    std::vector<int> stack{0};
    long long n = 0;
    while (!stack.empty()) {
        const int id = stack.back();
        stack.pop_back();
        if (id < 0 || id >= N) return fail_msg(HLGS_ERR_ARG, "node index out of range");
        const int* nd = nodes + 7 * (size_t)id;
        for (int i = 0; i < nd[3]; i++, n++)
            if (out && n < capacity) out[n] = nd[2] + i;
        if (nd[0] <= target) {
            for (int i = 0; i < nd[4]; i++, n++)
                if (out && n < capacity) out[n] = nd[2] + nd[3] + i;
        } else {
            for (int i = nd[6] - 1; i >= 0; i--) stack.push_back(nd[5] + i);
        }
    }
    if (n > 0x7fffffff) return fail_msg(HLGS_ERR_ARG, "expansion larger than 2^31 entries");
    *count = (int)n;
    return HLGS_OK;
}

}  // extern "C"
