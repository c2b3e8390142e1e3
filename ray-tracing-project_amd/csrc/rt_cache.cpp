// rt_cache.cpp -- binary scene cache: everything rt_scene_create derives from a mesh
// (object and world vertices, unit normals, plane distances, the reference's flat box partition with its face
// order, the traversal BVHs and triangle records), written once and reloaded without OBJ parsing or
// any build. The file is a versioned little-endian image of HostScene with a 64-bit content hash.
#include <chrono>
#include <cstdio>
#include <cstring>
#include <memory>
#include <utility>
#include <vector>

#include "rt_scene.h"

namespace {

constexpr char kMagic[8] = {'R', 'T', 'S', 'C', 'E', 'N', 'E', '1'};
// 2: + object-space vertices (RT_MODE_BOX_COLORS); 3: the header's builder field (version-2 files held 0
// there, which would read as RT_BUILDER_SAH whatever built them, so they are refused and rebuilt);
// 4: trees of scenes with tilted face normals bound the accept region (HostScene::av), not the world
// triangles, so an older file of such a scene could cull hits
constexpr uint32_t kVersion = 4;

struct Header {
  char magic[8];
  uint32_t version, header_bytes;
  int32_t nv, nf, n_mats, n_boxes, n_box_faces, n_nodes, n_nodes4, n_tris;
  uint32_t root;
  int32_t depth, leaves, depth4;
  int32_t min_faces, max_boxes, leaf_size, builder;  // builder: RT_BUILDER_* of the stored tree (was padding: 0)
  float M[16], Minv[16], MS[9], pad2[3];
};

struct BoxRec {  // RefBox without its face list
  float low[3], high[3], shape[3];
  uint8_t failed[3], pad;
  int32_t count;
};

// word-wise 64-bit content hash (multiply-xorshift; fast enough for a few hundred MB)
struct Hasher {
  uint64_t h = 0x9E3779B97F4A7C15ull;
  void add(const void* p, size_t n) {
    const unsigned char* b = static_cast<const unsigned char*>(p);
    size_t i = 0;
    for (; i + 8 <= n; i += 8) {
      uint64_t w;
      memcpy(&w, b + i, 8);
      h = (h ^ w) * 0xBF58476D1CE4E5B9ull;
      h ^= h >> 31;
    }
    uint64_t w = 0;
    memcpy(&w, b + i, n - i);
    h = (h ^ w ^ (uint64_t)n) * 0x94D049BB133111EBull;
    h ^= h >> 29;
  }
};

struct Writer {
  FILE* f;
  Hasher hash;
  bool ok = true;
  void put(const void* p, size_t n) {
    if (!n) return;
    hash.add(p, n);
    ok = ok && fwrite(p, 1, n, f) == n;
  }
  template <typename T>
  void vec(const std::vector<T>& v) { put(v.data(), v.size() * sizeof(T)); }
};

struct Reader {
  FILE* f;
  Hasher hash;
  bool ok = true;
  void get(void* p, size_t n) {
    if (!n) return;
    ok = ok && fread(p, 1, n, f) == n;
    if (ok) hash.add(p, n);
  }
  template <typename T>
  void vec(std::vector<T>& v, size_t n) {
    v.resize(n);
    get(v.data(), n * sizeof(T));
  }
};

}  // namespace

extern "C" int rt_scene_save(const rt_scene* s, const char* path) {
  if (!s || !path) { rt::set_error("rt_scene_save: null argument"); return RT_ERR_INVALID; }
  const rt::HostScene& hs = s->hs;
  std::unique_ptr<FILE, int (*)(FILE*)> fp(fopen(path, "wb"), fclose);
  if (!fp) { rt::set_error("rt_scene_save: cannot open %s", path); return RT_ERR_IO; }
  Header h;
  memset(&h, 0, sizeof h);
  memcpy(h.magic, kMagic, 8);
  h.version = kVersion;
  h.header_bytes = sizeof(Header);
  h.nv = hs.nv;
  h.nf = hs.nf;
  h.n_mats = (int32_t)hs.mats.size();
  h.n_boxes = (int32_t)hs.boxes.size();
  for (const rt::RefBox& b : hs.boxes) h.n_box_faces += (int32_t)b.faces.size();
  h.n_nodes = (int32_t)hs.nodes.size();
  h.n_nodes4 = (int32_t)hs.nodes4.size();
  h.n_tris = (int32_t)hs.tris.size();
  h.root = hs.root;
  h.depth = hs.depth;
  h.leaves = hs.leaves;
  h.depth4 = hs.depth4;
  h.min_faces = s->opts.min_faces;
  h.max_boxes = s->opts.max_boxes;
  h.leaf_size = s->opts.leaf_size;
  h.builder = s->builder_used;
  memcpy(h.M, hs.M, sizeof h.M);
  memcpy(h.Minv, hs.Minv, sizeof h.Minv);
  memcpy(h.MS, hs.MS, sizeof h.MS);
  Writer w{fp.get()};
  w.put(&h, sizeof h);
  w.vec(hs.wv);
  w.vec(hs.ov3);
  w.vec(hs.vnn);
  w.vec(hs.fnn);
  w.vec(hs.fdist);
  w.vec(hs.fidx);
  w.vec(hs.fmat);
  w.vec(hs.mats);
  std::vector<BoxRec> br(hs.boxes.size());
  std::vector<int32_t> bf;
  bf.reserve(h.n_box_faces);
  for (size_t i = 0; i < hs.boxes.size(); i++) {
    const rt::RefBox& b = hs.boxes[i];
    memset(&br[i], 0, sizeof br[i]);
    memcpy(br[i].low, b.low, 12);
    memcpy(br[i].high, b.high, 12);
    memcpy(br[i].shape, b.shape, 12);
    for (int k = 0; k < 3; k++) br[i].failed[k] = b.failed[k] ? 1 : 0;
    br[i].count = (int32_t)b.faces.size();
    bf.insert(bf.end(), b.faces.begin(), b.faces.end());
  }
  w.vec(br);
  w.vec(bf);
  w.vec(hs.face_rank);
  w.vec(hs.face_box);
  w.vec(hs.nodes);
  w.vec(hs.nodes4);
  w.vec(hs.tris);
  const uint64_t digest = w.hash.h;
  w.ok = w.ok && fwrite(&digest, 1, 8, fp.get()) == 8;
  if (!w.ok) { rt::set_error("rt_scene_save: write failed (%s)", path); return RT_ERR_IO; }
  return RT_OK;
}

extern "C" int rt_scene_load(const char* path, const rt_scene_opts* opts, rt_scene** out) {
  if (!path || !out) { rt::set_error("rt_scene_load: null argument"); return RT_ERR_INVALID; }
  *out = nullptr;
  auto t0 = std::chrono::steady_clock::now();
  std::unique_ptr<FILE, int (*)(FILE*)> fp(fopen(path, "rb"), fclose);
  if (!fp) { rt::set_error("rt_scene_load: cannot open %s", path); return RT_ERR_IO; }
  Header h;
  Reader r{fp.get()};
  r.get(&h, sizeof h);
  if (!r.ok || memcmp(h.magic, kMagic, 8) != 0 || h.version != kVersion || h.header_bytes != sizeof(Header)) {
    rt::set_error("rt_scene_load: %s is not a version-%u scene cache", path, kVersion);
    return RT_ERR_IO;
  }
  if (h.nv < 0 || h.nf < 0 || h.n_mats < 0 || h.n_boxes < 0 || h.n_box_faces != h.nf || h.n_nodes < 0 ||
      h.n_nodes4 < 0 || h.n_tris < h.nf || (uint32_t)h.n_tris > rt::kMaxFaces) {  // SBVH: references >= faces
    rt::set_error("rt_scene_load: inconsistent header in %s", path);
    return RT_ERR_IO;
  }
  std::unique_ptr<rt_scene> s(new rt_scene());
  if (opts) s->opts = *opts; else rt_scene_opts_default(&s->opts);
  // build parameters come from the cache (they shaped the stored boxes and BVH)
  s->opts.min_faces = h.min_faces;
  s->opts.max_boxes = h.max_boxes;
  s->opts.leaf_size = h.leaf_size;
  if (h.builder < RT_BUILDER_SAH || h.builder > RT_BUILDER_SBVH_GPU) { rt::set_error("rt_scene_load: bad builder id in %s", path); return RT_ERR_IO; }
  s->opts.builder = h.builder;
  s->builder_used = h.builder;
  s->opts.frames_in_flight = std::max(1, std::min(s->opts.frames_in_flight, (int32_t)rt_scene::kMaxSlots));
  rt::HostScene& hs = s->hs;
  hs.nv = h.nv;
  hs.nf = h.nf;
  hs.root = h.root;
  hs.depth = h.depth;
  hs.leaves = h.leaves;
  hs.depth4 = h.depth4;
  memcpy(hs.M, h.M, sizeof hs.M);
  memcpy(hs.Minv, h.Minv, sizeof hs.Minv);
  memcpy(hs.MS, h.MS, sizeof hs.MS);
  r.vec(hs.wv, h.nv);
  r.vec(hs.ov3, 3 * (size_t)h.nv);
  r.vec(hs.vnn, h.nv);
  r.vec(hs.fnn, h.nf);
  r.vec(hs.fdist, h.nf);
  r.vec(hs.fidx, 3 * (size_t)h.nf);
  r.vec(hs.fmat, h.nf);
  r.vec(hs.mats, h.n_mats);
  std::vector<BoxRec> br;
  std::vector<int32_t> bf;
  r.vec(br, h.n_boxes);
  r.vec(bf, h.n_box_faces);
  r.vec(hs.face_rank, h.nf);
  r.vec(hs.face_box, h.nf);
  r.vec(hs.nodes, h.n_nodes);
  r.vec(hs.nodes4, h.n_nodes4);
  r.vec(hs.tris, h.n_tris);
  uint64_t digest = 0;
  const uint64_t computed = r.hash.h;
  if (!r.ok || fread(&digest, 1, 8, fp.get()) != 8 || digest != computed) {
    rt::set_error("rt_scene_load: %s is truncated or corrupt", path);
    return RT_ERR_IO;
  }
  // reference boxes and index sanity (a cache must never make the kernels read out of bounds)
  hs.boxes.resize(h.n_boxes);
  size_t off = 0;
  for (int32_t i = 0; i < h.n_boxes; i++) {
    rt::RefBox& b = hs.boxes[i];
    memcpy(b.low, br[i].low, 12);
    memcpy(b.high, br[i].high, 12);
    memcpy(b.shape, br[i].shape, 12);
    for (int k = 0; k < 3; k++) b.failed[k] = br[i].failed[k] != 0;
    if (br[i].count < 0 || off + (size_t)br[i].count > bf.size()) { rt::set_error("rt_scene_load: bad box table"); return RT_ERR_IO; }
    b.faces.assign(bf.begin() + off, bf.begin() + off + br[i].count);
    off += br[i].count;
  }
  for (int32_t f = 0; f < h.nf; f++) {
    for (int k = 0; k < 3; k++)
      if (hs.fidx[3 * (size_t)f + k] >= (uint32_t)h.nv) { rt::set_error("rt_scene_load: bad face table"); return RT_ERR_IO; }
    if (hs.fmat[f] < -1 || hs.fmat[f] >= h.n_mats) { rt::set_error("rt_scene_load: bad material id"); return RT_ERR_IO; }
  }
  for (int32_t f = 0; f < h.nf; f++)
    if (hs.face_box[f] >= (uint32_t)h.n_boxes) { rt::set_error("rt_scene_load: bad face box"); return RT_ERR_IO; }
  for (const rt::TriRec64& t : hs.tris)
    if (t.face >= (uint32_t)h.nf || (t.box & rt::kBoxIndexMask) != hs.face_box[t.face]) {
      rt::set_error("rt_scene_load: bad triangle record");
      return RT_ERR_IO;
    }
  {
    // the records' flag bits let the kernels skip the normal check and the reference box predicate:
    // recomputed from the loaded geometry, never taken from the file (a crafted file could set them)
    const float Ro = rt::cert_origin_max(hs);
    rt::accept_region(hs);
    for (rt::TriRec64& t : hs.tris) t.box = (t.box & rt::kBoxIndexMask) | rt::tri_flags(hs, t.face, Ro);
  }
  auto handle_ok = [&](uint32_t c, int32_t n_inner) {
    if (rt::is_leaf(c)) return rt::leaf_first(c) + rt::leaf_count(c) <= (uint32_t)h.n_tris;
    return c < (uint32_t)n_inner;
  };
  for (const rt::Node64& n : hs.nodes)
    if (!handle_ok(n.child0, h.n_nodes) || !handle_ok(n.child1, h.n_nodes)) { rt::set_error("rt_scene_load: bad BVH"); return RT_ERR_IO; }
  for (const rt::Node4Q& n : hs.nodes4)
    for (int c = 0; c < 4; c++)
      if (((n.valid >> c) & 1) && !handle_ok(n.child[c], h.n_nodes4)) { rt::set_error("rt_scene_load: bad wide BVH"); return RT_ERR_IO; }
  // the root, whenever there are nodes (also for a face-less file: the tree walk below starts there)
  if ((h.nf > 0 || h.n_nodes > 0) && !handle_ok(h.root, h.n_nodes)) { rt::set_error("rt_scene_load: bad BVH root"); return RT_ERR_IO; }
  // Shape checks (the content hash is not a signature: a crafted file can carry a valid one). Each
  // tree must be a tree: walked from its root, every interior node is reached exactly once (no
  // cycle, no shared subtree), and its depth is recomputed here, never taken from the header, then
  // held to rt_scene_create's limits: the binary tree within the 64-entry wave stack, the wide tree
  // within kStack4 (else it is dropped and the binary traversal runs), and at most kMaxFaces faces
  // (32-bit byte offsets of the records).
  if ((uint32_t)h.nf > rt::kMaxFaces) { rt::set_error("rt_scene_load: %d faces exceed the %u-face limit", h.nf, rt::kMaxFaces); return RT_ERR_IO; }
  {
    std::vector<uint8_t> seen(hs.nodes.size(), 0);
    std::vector<std::pair<uint32_t, int>> st;
    int depth = 0;
    if (!hs.nodes.empty() && !rt::is_leaf(h.root)) st.push_back({h.root, 1});
    while (!st.empty()) {
      const auto [n, d] = st.back();
      st.pop_back();
      if (seen[n]++) { rt::set_error("rt_scene_load: BVH node %u reached twice (not a tree)", n); return RT_ERR_IO; }
      depth = std::max(depth, d + 1);
      if (depth > rt::kMaxDepth + 2) { rt::set_error("rt_scene_load: BVH deeper than the traversal stack"); return RT_ERR_IO; }
      const rt::Node64& nd = hs.nodes[n];
      if (!rt::is_leaf(nd.child1)) st.push_back({nd.child1, d + 1});
      if (!rt::is_leaf(nd.child0)) st.push_back({nd.child0, d + 1});
    }
    if (hs.nodes.empty() || rt::is_leaf(h.root)) {  // no interior node: nothing for the stack to hold
      if (h.depth < 0 || h.depth > 2) { rt::set_error("rt_scene_load: bad BVH depth"); return RT_ERR_IO; }
      hs.depth = h.depth;
    } else {
      hs.depth = depth;
    }
  }
  {
    std::vector<uint8_t> seen(hs.nodes4.size(), 0);
    std::vector<std::pair<uint32_t, int>> st;
    int maxd = -1;
    bool ok4 = true;
    if (!hs.nodes4.empty()) st.push_back({0u, 0});
    while (!st.empty() && ok4) {
      const auto [n, d] = st.back();
      st.pop_back();
      if (seen[n]++) { ok4 = false; break; }
      maxd = std::max(maxd, d);
      if (3 * (maxd + 1) + 4 > rt::kStack4) { ok4 = false; break; }
      const rt::Node4Q& nd = hs.nodes4[n];
      for (int c = 0; c < 4; c++)
        if (((nd.valid >> c) & 1) && !rt::is_leaf(nd.child[c])) st.push_back({nd.child[c], d + 1});
    }
    if (!ok4) {  // not a tree or too deep for the wide stack: keep the binary traversal only
      hs.nodes4.clear();
      hs.depth4 = 0;
    } else {
      hs.depth4 = hs.nodes4.empty() ? 0 : maxd + 1;
    }
  }
  if (s->opts.wide_tree) rt::build_wide(hs);  // derived from the validated binary tree (not stored)
  s->build_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  if (s->opts.device != RT_DEVICE_NONE) {
    int rc = rt::resolve_devices(s->opts);
    if (rc) return rc;
    if ((rc = rt::device_upload(s.get()))) return rc;
    if (s->opts.n_devices > 1 && (rc = rt::device_replicate(s.get()))) return rc;
  } else if (s->opts.n_devices != 0) {
    rt::set_error("rt_scene_load: a host-only scene (RT_DEVICE_NONE) lists no devices");
    return RT_ERR_INVALID;
  }
  *out = s.release();
  return RT_OK;
}
