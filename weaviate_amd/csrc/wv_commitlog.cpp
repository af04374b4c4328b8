// wv_commitlog.cpp -- HNSW commit log -> fixed-degree CSR loader (host C++).
//
// A Weaviate shard persists its graph as a write-ahead log of typed records
// (adapters/repos/db/vector/hnsw/commitlog/logger.go:28-215), condensed and
// combined in the background, and replayed at startup by Deserializer.Do
// (deserializer.go:80-158) over every log file in timestamp order
// (startup.go:56-152, getCommitFileNames commit_logger.go:121-166).  This file
// replays the same records into the same state and exports it as the CSR the
// GPU searches (wvgpu.h wv_index_upload_graph), so a GPU mirror can serve an
// existing shard without rebuilding its graph.  Read-only: unlike the
// reference it never truncates or deletes a file; a torn tail is reported.
#include <dirent.h>

#include <algorithm>
#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <unordered_set>
#include <vector>

#include "../../include/wvgpu.h"

extern "C" void wv_internal_set_error(const char* msg);

namespace {

enum : uint8_t {
    AddNode = 0, SetEntryPointMaxLevel, AddLinkAtLevel, ReplaceLinksAtLevel, AddTombstone, RemoveTombstone,
    ClearLinks, DeleteNode, ResetIndex, ClearLinksAtLevel, AddLinksAtLevel, AddPQ
};

constexpr uint64_t kMaxId = (1ull << 32) - 2;   // the GPU holds uint32 local ids

struct Vertex {
    int level = 0;
    std::vector<std::vector<uint64_t>> conns;
};

int fail(int code, const std::string& m) {
    wv_internal_set_error(m.c_str());
    return code;
}

struct Reader {
    const uint8_t* p;
    size_t n, off = 0;
    bool get(void* dst, size_t k) {
        if (off + k > n) { off = n; return false; }
        std::memcpy(dst, p + off, k);
        off += k;
        return true;
    }
    bool u8(uint8_t& v) { return get(&v, 1); }
    bool u16(uint16_t& v) {
        uint8_t b[2];
        if (!get(b, 2)) return false;
        v = (uint16_t)(b[0] | (b[1] << 8));
        return true;
    }
    bool u64(uint64_t& v) {
        uint8_t b[8];
        if (!get(b, 8)) return false;
        v = 0;
        for (int i = 7; i >= 0; --i) v = (v << 8) | b[i];
        return true;
    }
    bool skip(size_t k) {
        if (off + k > n) { off = n; return false; }
        off += k;
        return true;
    }
};

}  // namespace

struct wv_graph {
    std::vector<Vertex*> nodes;   // nullptr = nil node
    std::unordered_set<uint64_t> tombstones;
    uint64_t entrypoint = 0;
    uint16_t level = 0;
    bool compressed = false;
    // the last AddPQ record's quantizer (ReadPQ :510-563): header and, for the
    // KMeans encoder, every segment's Ks x dims/M centres (ReadKMeansEncoder
    // :487-508, little-endian float32, ExposeDataForRestore's order)
    uint16_t pq_dims = 0, pq_ks = 0, pq_m = 0;
    uint8_t pq_enc = 0, pq_dist = 0, pq_bits = 0;
    std::vector<float> pq_centers;
    bool truncated = false;       // a file ended inside a record
    uint64_t valid_bytes = 0;     // bytes of complete records, all files
    uint64_t dropped_links = 0;   // export: links to ids past the last node

    ~wv_graph() { clear_nodes(); }
    void clear_nodes() {
        for (Vertex* v : nodes) delete v;
        nodes.clear();
    }
    // growIndexToAccomodateNode: the node array covers id
    bool grow(uint64_t id) {
        if (id > kMaxId) return false;
        if (id >= nodes.size()) nodes.resize(id + 1, nullptr);
        return true;
    }
    static void grow_levels(Vertex* v, uint16_t level) {   // maybeGrowConnectionsForLevel
        if (v->conns.size() <= level) v->conns.resize((size_t)level + 1);
    }
    Vertex* node_for_link(uint64_t id, uint16_t level) {   // ReadLink / ReadLinks / ReadAddLinks
        Vertex*& v = nodes[id];
        if (!v) {
            v = new Vertex();
            v->conns.resize((size_t)level + 1);
        }
        grow_levels(v, level);
        return v;
    }

    // Deserializer.Do over one file (deserializer.go:80-158).  Returns WV_OK
    // (including a torn tail: state keeps every complete record) or an error
    // for an unknown record type / an id beyond the GPU's range.
    int replay(const uint8_t* buf, size_t len) {
        Reader r{buf, len};
        std::vector<uint64_t> tg;
        for (;;) {
            const size_t start = r.off;
            uint8_t ct;
            if (!r.u8(ct)) break;   // clean EOF
            uint64_t id = 0, target = 0;
            uint16_t lv = 0, cnt = 0;
            bool ok = true;
            switch (ct) {
            case AddNode:   // ReadNode :160-187
                ok = r.u64(id) && r.u16(lv);
                if (ok) {
                    if (!grow(id)) return fail(WV_EINVAL, "commit log: node id beyond the GPU id range");
                    Vertex*& v = nodes[id];
                    if (!v) {
                        v = new Vertex();
                        v->level = lv;
                        v->conns.resize((size_t)lv + 1);
                    } else {
                        grow_levels(v, lv);
                        v->level = lv;
                    }
                }
                break;
            case SetEntryPointMaxLevel:   // ReadEP :189-201
                ok = r.u64(id) && r.u16(lv);
                if (ok) { entrypoint = id; level = lv; }
                break;
            case AddLinkAtLevel:   // ReadLink :203-236
                ok = r.u64(id) && r.u16(lv) && r.u64(target);
                if (ok) {
                    if (!grow(id)) return fail(WV_EINVAL, "commit log: node id beyond the GPU id range");
                    node_for_link(id, lv)->conns[lv].push_back(target);
                }
                break;
            case ReplaceLinksAtLevel:   // ReadLinks :238-285
            case AddLinksAtLevel: {     // ReadAddLinks :287-324
                ok = r.u64(id) && r.u16(lv) && r.u16(cnt);
                tg.resize(cnt);
                for (uint16_t i = 0; ok && i < cnt; ++i) ok = r.u64(tg[i]);
                if (ok) {
                    if (!grow(id)) return fail(WV_EINVAL, "commit log: node id beyond the GPU id range");
                    std::vector<uint64_t>& c = node_for_link(id, lv)->conns[lv];
                    if (ct == ReplaceLinksAtLevel) c.assign(tg.begin(), tg.end());
                    else c.insert(c.end(), tg.begin(), tg.end());
                }
                break;
            }
            case AddTombstone:   // :326-335
                ok = r.u64(id);
                if (ok) tombstones.insert(id);
                break;
            case RemoveTombstone:   // :337-346
                ok = r.u64(id);
                if (ok) tombstones.erase(id);
                break;
            case ClearLinks:   // ReadClearLinks :348-368
                ok = r.u64(id);
                if (ok && id < nodes.size() && nodes[id]) {
                    const size_t nl = nodes[id]->conns.size();
                    nodes[id]->conns.assign(nl, {});
                }
                break;
            case ClearLinksAtLevel:   // ReadClearLinksAtLevel :370-434, keepReplaceInfo = false at startup
                ok = r.u64(id) && r.u16(lv);
                if (ok && id < nodes.size() && nodes[id]) {
                    Vertex* v = nodes[id];
                    if (v->conns.empty()) {
                        v->conns.resize((size_t)lv + 1);
                    } else {
                        grow_levels(v, lv);
                        v->conns[lv].clear();
                    }
                }
                break;
            case DeleteNode:   // ReadDeleteNode :436-449
                ok = r.u64(id);
                if (ok && id < nodes.size()) {
                    delete nodes[id];
                    nodes[id] = nullptr;
                }
                break;
            case ResetIndex:   // :139-142 (tombstones survive)
                entrypoint = 0;
                level = 0;
                clear_nodes();
                break;
            case AddPQ: {   // ReadPQ :510-563
                uint16_t dims = 0, ks = 0, m = 0;
                uint8_t enc = 0, dist = 0, bits = 0;
                ok = r.u16(dims) && r.u8(enc) && r.u16(ks) && r.u16(m) && r.u8(dist) && r.u8(bits);
                std::vector<float> centers;
                for (uint16_t i = 0; ok && i < m; ++i) {
                    // ssdhelpers: UseTileEncoder = 0 (51 bytes, tile_encoder.go:138-149),
                    // UseKMeansEncoder = 1 (Ks x dims/M float32 centres, kmeans.go:61-69)
                    if (enc == 0) {
                        ok = r.skip(6 * 8 + 2 + 1);
                    } else if (enc == 1) {
                        const size_t nf = (size_t)ks * (dims / (m ? m : 1));
                        const size_t at = centers.size();
                        centers.resize(at + nf);
                        for (size_t j = 0; ok && j < nf; ++j) {
                            uint8_t b[4];
                            ok = r.get(b, 4);
                            const uint32_t u = (uint32_t)b[0] | (uint32_t)b[1] << 8 | (uint32_t)b[2] << 16 |
                                               (uint32_t)b[3] << 24;
                            std::memcpy(&centers[at + j], &u, 4);
                        }
                    } else {
                        return fail(WV_EINVAL, "commit log: unsupported PQ encoder type");
                    }
                }
                if (ok) {
                    compressed = true;
                    pq_dims = dims; pq_ks = ks; pq_m = m; pq_enc = enc; pq_dist = dist; pq_bits = bits;
                    pq_centers.swap(centers);
                }
                break;
            }
            default:
                return fail(WV_EINVAL, "commit log: unrecognized commit type " + std::to_string(ct));
            }
            if (!ok) {   // torn record: startup.go:93-107 keeps the valid prefix
                truncated = true;
                (void)start;
                break;
            }
            valid_bytes += r.off - start;
        }
        return WV_OK;
    }
};

namespace {

int read_file(const std::string& path, std::vector<uint8_t>& out) {
    FILE* f = std::fopen(path.c_str(), "rb");
    if (!f) return fail(WV_EINVAL, "open commit log " + path + ": " + std::strerror(errno));
    out.clear();
    uint8_t buf[1 << 16];
    size_t k;
    while ((k = std::fread(buf, 1, sizeof buf, f)) > 0) out.insert(out.end(), buf, buf + k);
    std::fclose(f);
    return WV_OK;
}

bool ends_with(const std::string& s, const std::string& suf) {
    return s.size() >= suf.size() && s.compare(s.size() - suf.size(), suf.size(), suf) == 0;
}

}  // namespace

extern "C" {

int wv_graph_load_commitlog_buffer(const uint8_t* buf, uint64_t len, wv_graph** out) {
    if (!out || (!buf && len)) return fail(WV_EINVAL, "wv_graph_load_commitlog_buffer: bad argument");
    auto* g = new wv_graph();
    const int rc = g->replay(buf, len);
    if (rc) { delete g; return rc; }
    *out = g;
    return WV_OK;
}

int wv_graph_load_commitlogs(const char* const* paths, int n_paths, wv_graph** out) {
    if (!out || n_paths < 0 || (n_paths && !paths)) return fail(WV_EINVAL, "wv_graph_load_commitlogs: bad argument");
    auto* g = new wv_graph();
    std::vector<uint8_t> data;
    for (int i = 0; i < n_paths; ++i) {
        int rc = read_file(paths[i], data);
        if (!rc) rc = g->replay(data.data(), data.size());
        if (rc) { delete g; return rc; }
    }
    *out = g;
    return WV_OK;
}

int wv_graph_load_commitlog_dir(const char* dir, wv_graph** out) {
    if (!dir || !out) return fail(WV_EINVAL, "wv_graph_load_commitlog_dir: bad argument");
    DIR* d = opendir(dir);
    if (!d) return fail(WV_EINVAL, std::string("open commit log directory ") + dir + ": " + std::strerror(errno));
    std::vector<std::string> names;
    while (dirent* e = readdir(d)) {
        const std::string n = e->d_name;
        // removeTmpScratchOrHiddenFiles / removeTmpCombiningFiles (commit_logger.go:206-249)
        if (n.empty() || n[0] == '.' || ends_with(n, ".scratch.tmp") || ends_with(n, ".combined.tmp")) continue;
        names.push_back(n);
    }
    closedir(d);
    // CorruptCommitLogFixer (corrupt_commit_logs_fixer.go:43-70): a .condensed
    // file whose original still exists is an interrupted condense -- skipped
    std::vector<std::string> keep;
    for (const std::string& n : names) {
        if (ends_with(n, ".condensed") &&
            std::find(names.begin(), names.end(), n.substr(0, n.size() - 10)) != names.end())
            continue;
        keep.push_back(n);
    }
    // asTimeStamp ordering (commit_logger.go:144-155, 251-253)
    std::vector<std::pair<long long, std::string>> ts;
    for (const std::string& n : keep) {
        const std::string base = ends_with(n, ".condensed") ? n.substr(0, n.size() - 10) : n;
        char* endp = nullptr;
        errno = 0;
        const long long t = std::strtoll(base.c_str(), &endp, 10);
        if (errno || !endp || *endp != '\0' || base.empty())
            return fail(WV_EINVAL, "commit log file name is not a timestamp: " + n);
        ts.emplace_back(t, n);
    }
    std::stable_sort(ts.begin(), ts.end(), [](const auto& a, const auto& b) { return a.first < b.first; });
    std::vector<std::string> paths;
    for (auto& t : ts) paths.push_back(std::string(dir) + "/" + t.second);
    std::vector<const char*> pp;
    for (auto& p : paths) pp.push_back(p.c_str());
    return wv_graph_load_commitlogs(pp.data(), (int)pp.size(), out);
}

int wv_graph_get_info(const wv_graph* g, wv_graph_info* info) {
    if (!g || !info) return fail(WV_EINVAL, "wv_graph_get_info: bad argument");
    std::memset(info, 0, sizeof(*info));
    uint64_t n = 0, up = 0;
    int md0 = 0, mdu = 0, ml = 0;
    for (uint64_t i = 0; i < g->nodes.size(); ++i) {
        const Vertex* v = g->nodes[i];
        if (!v) continue;
        n = i + 1;
        if (v->level >= 1) up++;
        ml = std::max(ml, v->level);
        if (!v->conns.empty()) md0 = std::max(md0, (int)v->conns[0].size());
        for (int l = 1; l <= v->level && l < (int)v->conns.size(); ++l) mdu = std::max(mdu, (int)v->conns[l].size());
    }
    info->n_slots = n;
    info->entrypoint = g->entrypoint;
    info->max_level = g->level;
    info->max_node_level = ml;
    info->n_upper = up;
    info->n_tombstones = g->tombstones.size();
    info->max_deg0 = md0;
    info->max_degU = mdu;
    info->compressed = g->compressed;
    info->truncated = g->truncated;
    info->valid_bytes = g->valid_bytes;
    return WV_OK;
}

int wv_graph_node(const wv_graph* g, uint64_t id, int level, int* node_level, uint64_t* links, int cap, int* n_links) {
    if (!g || !node_level || !n_links) return fail(WV_EINVAL, "wv_graph_node: bad argument");
    *n_links = 0;
    if (id >= g->nodes.size() || !g->nodes[id]) { *node_level = -1; return WV_OK; }
    const Vertex* v = g->nodes[id];
    *node_level = v->level;
    if (level < 0 || level >= (int)v->conns.size()) return WV_OK;
    const auto& c = v->conns[level];
    *n_links = (int)c.size();
    for (int i = 0; i < (int)c.size() && i < cap; ++i) links[i] = c[i];
    return WV_OK;
}

int wv_graph_export_csr(wv_graph* g, int deg0, int degU, int8_t* levels, uint32_t* layer0, uint32_t* upper_row,
                        uint32_t* upper, uint64_t* tomb_bits) {
    wv_graph_info info;
    if (!g || deg0 <= 0 || degU <= 0 || !levels || !layer0 || !upper_row || !upper)
        return fail(WV_EINVAL, "wv_graph_export_csr: bad argument");
    wv_graph_get_info(g, &info);
    if (info.max_deg0 > deg0 || info.max_degU > degU)
        return fail(WV_EINVAL, "wv_graph_export_csr: a neighbour list is longer than the CSR degree");
    const uint64_t n = info.n_slots;
    const int ml = std::max(1, info.max_node_level);
    uint64_t row = 0, dropped = 0;
    for (uint64_t i = 0; i < n; ++i) {
        const Vertex* v = g->nodes[i];
        uint32_t* r0 = layer0 + i * (uint64_t)deg0;
        std::fill(r0, r0 + deg0, 0xFFFFFFFFu);
        levels[i] = v ? (int8_t)std::min(v->level, 127) : (int8_t)-1;
        upper_row[i] = 0xFFFFFFFFu;
        if (!v) continue;
        // links to ids past the last node cannot be searched (their vector
        // lookup fails, search.go:420-458): dropped
        auto put = [&](uint32_t* dst, int cap, const std::vector<uint64_t>& c) {
            int k = 0;
            for (uint64_t t : c) {
                if (t >= n) { dropped++; continue; }
                if (k < cap) dst[k++] = (uint32_t)t;
            }
        };
        if (!v->conns.empty()) put(r0, deg0, v->conns[0]);
        if (v->level >= 1) {
            upper_row[i] = (uint32_t)row;
            for (int l = 1; l <= ml; ++l) {
                uint32_t* ru = upper + (row * (uint64_t)ml + (l - 1)) * degU;
                std::fill(ru, ru + degU, 0xFFFFFFFFu);
                if (l <= v->level && l < (int)v->conns.size()) put(ru, degU, v->conns[l]);
            }
            row++;
        }
    }
    g->dropped_links = dropped;
    if (tomb_bits) {
        std::fill(tomb_bits, tomb_bits + (n + 63) / 64, 0ull);
        for (uint64_t t : g->tombstones)
            if (t < n) tomb_bits[t >> 6] |= 1ull << (t & 63);
    }
    return WV_OK;
}

int wv_graph_get_pq(const wv_graph* g, wv_graph_pq* pq, float* centroid_table, uint64_t table_cap) {
    if (!g || !pq) return fail(WV_EINVAL, "wv_graph_get_pq: bad argument");
    std::memset(pq, 0, sizeof(*pq));
    if (!g->compressed) return WV_OK;
    pq->present = 1;
    pq->dims = g->pq_dims;
    pq->segments = g->pq_m;
    pq->centroids = g->pq_ks;
    pq->encoder = g->pq_enc;
    pq->distribution = g->pq_dist;
    pq->use_bits_encoding = g->pq_bits;
    pq->table_floats = g->pq_centers.size();
    if (centroid_table && table_cap >= g->pq_centers.size())
        std::memcpy(centroid_table, g->pq_centers.data(), g->pq_centers.size() * sizeof(float));
    return WV_OK;
}

int wv_graph_destroy(wv_graph* g) {
    delete g;
    return WV_OK;
}

}  // extern "C"
