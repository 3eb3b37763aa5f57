// cgltrace.cpp -- boost-XML-archive subset reader for .cgltrace scenes.
// See cgltrace.h for provenance.  A small DOM (element name, text, children)
// is built in one pass; gzip-compressed files are inflated with zlib.
#include "cgltrace.h"

#include <zlib.h>

#include <cctype>
#include <cstdlib>
#include <cstring>
#include <memory>

namespace rt {
namespace {

struct Node {
  std::string name;
  std::string text;
  std::vector<std::unique_ptr<Node>> kids;

  const Node* child(const char* n) const {
    for (auto& k : kids)
      if (k->name == n) return k.get();
    return nullptr;
  }
};

bool read_all(const std::string& path, std::string* out) {
  gzFile f = gzopen(path.c_str(), "rb");  // transparently reads plain files too
  if (!f) return false;
  char buf[1 << 16];
  int n;
  while ((n = gzread(f, buf, sizeof(buf))) > 0) out->append(buf, (size_t)n);
  const bool ok = (n == 0);
  gzclose(f);
  return ok;
}

// Minimal XML: elements, attributes (ignored), text, <?...?>, <!...>, comments.
class Parser {
 public:
  explicit Parser(const std::string& s) : s_(s) {}

  std::unique_ptr<Node> parse(std::string* err) {
    auto root = std::make_unique<Node>();
    root->name = "#document";
    std::vector<Node*> stack{root.get()};
    while (i_ < s_.size()) {
      if (s_[i_] != '<') {
        const size_t j = s_.find('<', i_);
        const size_t e = (j == std::string::npos) ? s_.size() : j;
        stack.back()->text.append(s_, i_, e - i_);
        i_ = e;
        continue;
      }
      if (s_.compare(i_, 4, "<!--") == 0) {
        const size_t j = s_.find("-->", i_);
        if (j == std::string::npos) return fail(err, "unterminated comment");
        i_ = j + 3;
        continue;
      }
      if (s_.compare(i_, 2, "<?") == 0 || s_.compare(i_, 2, "<!") == 0) {
        const size_t j = s_.find('>', i_);
        if (j == std::string::npos) return fail(err, "unterminated declaration");
        i_ = j + 1;
        continue;
      }
      const size_t j = s_.find('>', i_);
      if (j == std::string::npos) return fail(err, "unterminated tag");
      if (s_[i_ + 1] == '/') {  // closing tag
        const std::string name = tag_name(i_ + 2, j);
        if (stack.size() < 2 || stack.back()->name != name)
          return fail(err, "mismatched closing tag </" + name + ">");
        stack.pop_back();
        i_ = j + 1;
        continue;
      }
      const bool self_close = s_[j - 1] == '/';
      auto node = std::make_unique<Node>();
      node->name = tag_name(i_ + 1, self_close ? j - 1 : j);
      Node* raw = node.get();
      stack.back()->kids.push_back(std::move(node));
      if (!self_close) stack.push_back(raw);
      i_ = j + 1;
    }
    if (stack.size() != 1) return fail(err, "unexpected end of document");
    return root;
  }

 private:
  std::string tag_name(size_t b, size_t e) const {
    size_t k = b;
    while (k < e && !std::isspace((unsigned char)s_[k])) ++k;
    return s_.substr(b, k - b);
  }
  std::unique_ptr<Node> fail(std::string* err, const std::string& m) {
    if (err) *err = m + " at byte " + std::to_string(i_);
    return nullptr;
  }
  const std::string& s_;
  size_t i_ = 0;
};

bool get_int(const Node* n, const char* name, int64_t* v) {
  const Node* c = n ? n->child(name) : nullptr;
  if (!c) return false;
  *v = std::strtoll(c->text.c_str(), nullptr, 10);
  return true;
}
bool get_float(const Node* n, const char* name, float* v) {
  const Node* c = n ? n->child(name) : nullptr;
  if (!c) return false;
  *v = std::strtof(c->text.c_str(), nullptr);  // correctly rounded decimal -> fp32
  return true;
}

bool base64_decode(const std::string& in, std::vector<uint8_t>* out) {
  static int8_t tbl[256];
  static bool init = false;
  if (!init) {
    std::memset(tbl, -1, sizeof(tbl));
    const char* a = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/";
    for (int i = 0; i < 64; ++i) tbl[(uint8_t)a[i]] = (int8_t)i;
    init = true;
  }
  uint32_t acc = 0;
  int bits = 0;
  for (unsigned char ch : in) {
    if (std::isspace(ch)) continue;
    if (ch == '=') break;
    const int v = tbl[ch];
    if (v < 0) return false;
    acc = (acc << 6) | (uint32_t)v;
    bits += 6;
    if (bits >= 8) {
      bits -= 8;
      out->push_back((uint8_t)((acc >> bits) & 0xff));
    }
  }
  return true;
}

}  // namespace

int LoadCGLTrace(const std::string& path, Scene* scene, std::string* error) {
  std::string xml;
  if (!read_all(path, &xml)) {
    if (error) *error = "cannot read " + path;
    return -1;
  }
  std::string err;
  auto doc = Parser(xml).parse(&err);
  auto bad = [&](const std::string& m) {
    if (error) *error = path + ": " + m;
    return -1;
  };
  if (!doc) return bad(err);
  const Node* arch = doc->child("boost_serialization");
  const Node* cgl = arch ? arch->child("cgltrace") : doc->child("cgltrace");
  if (!cgl) return bad("no <cgltrace> element");
  const Node* dcs = cgl->child("drawcalls");
  if (!dcs) return bad("no <drawcalls>");
  *scene = Scene();
  for (auto& item : dcs->kids) {
    if (item->name != "item") continue;
    DrawCall dc;
    const Node* st = item->child("states");
    if (!st) return bad("drawcall without <states>");
    int64_t v = 0;
#define ST(f) \
  if (get_int(st, #f, &v)) dc.states.f = (decltype(dc.states.f))v;
    ST(color_enabled) ST(color_format) ST(color_writemask) ST(depth_test) ST(depth_writemask)
    ST(depth_format) ST(depth_func) ST(stencil_test) ST(stencil_func) ST(stencil_zpass)
    ST(stencil_zfail) ST(stencil_fail) ST(stencil_ref) ST(stencil_mask) ST(stencil_writemask)
    ST(texture_enabled) ST(texture_envmode) ST(texture_minfilter) ST(texture_magfilter)
    ST(texture_addressU) ST(texture_addressV) ST(blend_enabled) ST(blend_src) ST(blend_dst)
#undef ST
    if (get_int(item.get(), "texture_id", &v)) dc.texture_id = (int32_t)v;
    std::map<int64_t, Vertex> verts;
    if (const Node* vs = item->child("vertices")) {
      for (auto& vi : vs->kids) {
        if (vi->name != "item") continue;
        int64_t id = 0;
        const Node* sec = vi->child("second");
        if (!get_int(vi.get(), "first", &id) || !sec) return bad("bad vertex entry");
        Vertex vx{};
        const Node* pos = sec->child("pos");
        const Node* col = sec->child("color");
        const Node* tc = sec->child("texcoord");
        if (!pos || !col || !tc) return bad("vertex without pos/color/texcoord");
        get_float(pos, "x", &vx.pos[0]); get_float(pos, "y", &vx.pos[1]);
        get_float(pos, "z", &vx.pos[2]); get_float(pos, "w", &vx.pos[3]);
        get_float(col, "r", &vx.color[0]); get_float(col, "g", &vx.color[1]);
        get_float(col, "b", &vx.color[2]); get_float(col, "a", &vx.color[3]);
        get_float(tc, "u", &vx.uv[0]); get_float(tc, "v", &vx.uv[1]);
        verts[id] = vx;
      }
    }
    dc.prim_offset = (uint32_t)scene->prims.size();
    if (const Node* ps = item->child("primitives")) {
      for (auto& pi : ps->kids) {
        if (pi->name != "item") continue;
        int64_t i0, i1, i2;
        if (!get_int(pi.get(), "i0", &i0) || !get_int(pi.get(), "i1", &i1) ||
            !get_int(pi.get(), "i2", &i2))
          return bad("bad primitive entry");
        auto f0 = verts.find(i0), f1 = verts.find(i1), f2 = verts.find(i2);
        if (f0 == verts.end() || f1 == verts.end() || f2 == verts.end())
          return bad("primitive references a missing vertex");
        scene->prims.push_back({f0->second, f1->second, f2->second});
      }
    }
    dc.prim_count = (uint32_t)scene->prims.size() - dc.prim_offset;
    if (const Node* vp = item->child("viewport")) {
      const char* k[6] = {"left", "right", "top", "bottom", "near", "far"};
      for (int i = 0; i < 6; ++i) get_float(vp, k[i], &dc.viewport[i]);
    }
    scene->drawcalls.push_back(dc);
  }
  if (const Node* ts = cgl->child("textures")) {
    for (auto& ti : ts->kids) {
      if (ti->name != "item") continue;
      int64_t id = 0, fmt = 0, w = 0, h = 0, size = -1;
      const Node* sec = ti->child("second");
      if (!get_int(ti.get(), "first", &id) || !sec) return bad("bad texture entry");
      get_int(sec, "format", &fmt);
      get_int(sec, "width", &w);
      get_int(sec, "height", &h);
      get_int(sec, "size", &size);
      Texture t;
      t.format = (int32_t)fmt;
      t.width = (int32_t)w;
      t.height = (int32_t)h;
      const Node* px = sec->child("pixels");
      if (px && !base64_decode(px->text, &t.pixels)) return bad("bad base64 texel data");
      if (size >= 0 && (int64_t)t.pixels.size() != size) return bad("texture size mismatch");
      scene->textures[(int32_t)id] = std::move(t);
    }
  }
  return 0;
}

}  // namespace rt
