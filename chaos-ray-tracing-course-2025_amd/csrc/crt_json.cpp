/*
 * crt_json.cpp — .crtscene loader (host C++), replacing
 *   crt::json::read_scene_from_istream   src/core/crt_json.cpp:541-647
 * whose rapidjson dependency (vendor/rapidjson, an un-checked-out submodule,
 * .gitmodules:4-6) is absent.  The DOM parser below is written from scratch and
 * reproduces what the loader observes of rapidjson's default (non full-
 * precision) reader: the IsInt/IsNumber typing of numbers and the double value
 * produced by its normal-precision path (integer significand in uint64, then
 * one multiply/divide by an exactly-rounded power of ten), narrowed with
 * GetFloat() = static_cast<float>(GetDouble()).
 *
 * Accept/reject rules, defaults and quirks follow crt_json.cpp line by line;
 * deviations (the reference would read out of bounds / invoke UB) are marked
 * "UB in reference".
 */
#include <cmath>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <limits>
#include <memory>
#include <sstream>
#include <string>
#include <unordered_map>
#include <vector>

#include "crt_host.h"

namespace crt_amd {
namespace json {

/* ---------------------------------------------------------------------- */
/*  minimal DOM                                                            */
/* ---------------------------------------------------------------------- */
enum class Kind { Null, False, True, Number, String, Array, Object };

struct Value {
    Kind kind = Kind::Null;
    /* numbers: rapidjson's type flags (document.h kIntFlag … kDoubleFlag) */
    bool is_int = false, is_double = false;
    double num = 0.0;
    std::string str;
    std::vector<Value> items;                                  /* array */
    std::vector<std::pair<std::string, Value>> members;        /* object, in file order */

    bool IsArray() const { return kind == Kind::Array; }
    bool IsObject() const { return kind == Kind::Object; }
    bool IsString() const { return kind == Kind::String; }
    bool IsBool() const { return kind == Kind::True || kind == Kind::False; }
    bool GetBool() const { return kind == Kind::True; }
    bool IsNumber() const { return kind == Kind::Number; }
    bool IsInt() const { return kind == Kind::Number && is_int; }
    int GetInt() const { return (int)num; }
    float GetFloat() const { return static_cast<float>(num); }
    size_t Size() const { return items.size(); }
    /* FindMember: linear search, first match wins (rapidjson document.h). */
    const Value *Find(const char *name) const {
        for (const auto &m : members)
            if (m.first == name) return &m.second;
        return nullptr;
    }
    bool Equals(const char *s) const { return kind == Kind::String && str == s; }
};

class Parser {
public:
    Parser(const char *p, size_t n) : s_(p), e_(p + n) {}

    bool parse_document(Value &out) {
        ws();
        if (!value(out, 0)) return false;
        ws();
        return s_ == e_;   /* kParseErrorDocumentRootNotSingular otherwise */
    }

private:
    const char *s_, *e_;

    char peek() const { return s_ < e_ ? *s_ : '\0'; }
    void ws() { while (s_ < e_ && (*s_ == ' ' || *s_ == '\n' || *s_ == '\r' || *s_ == '\t')) ++s_; }
    bool lit(const char *w) {
        const size_t n = std::strlen(w);
        if ((size_t)(e_ - s_) < n || std::memcmp(s_, w, n) != 0) return false;
        s_ += n;
        return true;
    }

    bool value(Value &v, int depth) {
        if (depth > 512) return false;
        switch (peek()) {
        case 'n': v.kind = Kind::Null; return lit("null");
        case 't': v.kind = Kind::True; return lit("true");
        case 'f': v.kind = Kind::False; return lit("false");
        case '"': v.kind = Kind::String; return string(v.str);
        case '[': return array(v, depth);
        case '{': return object(v, depth);
        default: v.kind = Kind::Number; return number(v);
        }
    }

    static void put_utf8(std::string &o, unsigned cp) {
        if (cp < 0x80) o += (char)cp;
        else if (cp < 0x800) { o += (char)(0xC0 | (cp >> 6)); o += (char)(0x80 | (cp & 0x3F)); }
        else if (cp < 0x10000) {
            o += (char)(0xE0 | (cp >> 12)); o += (char)(0x80 | ((cp >> 6) & 0x3F)); o += (char)(0x80 | (cp & 0x3F));
        } else {
            o += (char)(0xF0 | (cp >> 18)); o += (char)(0x80 | ((cp >> 12) & 0x3F));
            o += (char)(0x80 | ((cp >> 6) & 0x3F)); o += (char)(0x80 | (cp & 0x3F));
        }
    }
    bool hex4(unsigned &cp) {
        cp = 0;
        for (int i = 0; i < 4; ++i) {
            const char c = peek();
            ++s_;
            cp <<= 4;
            if (c >= '0' && c <= '9') cp |= (unsigned)(c - '0');
            else if (c >= 'a' && c <= 'f') cp |= (unsigned)(c - 'a' + 10);
            else if (c >= 'A' && c <= 'F') cp |= (unsigned)(c - 'A' + 10);
            else return false;
        }
        return true;
    }
    bool string(std::string &o) {
        ++s_;  /* opening quote */
        for (;;) {
            if (s_ >= e_) return false;
            const unsigned char c = (unsigned char)*s_++;
            if (c == '"') return true;
            if (c < 0x20) return false;   /* kParseErrorStringInvalidEncoding / control char */
            if (c != '\\') { o += (char)c; continue; }
            const char x = peek();
            ++s_;
            switch (x) {
            case '"': o += '"'; break;
            case '\\': o += '\\'; break;
            case '/': o += '/'; break;
            case 'b': o += '\b'; break;
            case 'f': o += '\f'; break;
            case 'n': o += '\n'; break;
            case 'r': o += '\r'; break;
            case 't': o += '\t'; break;
            case 'u': {
                unsigned cp;
                if (!hex4(cp)) return false;
                if (cp >= 0xD800 && cp <= 0xDBFF) {
                    if (!(peek() == '\\')) return false;
                    ++s_;
                    if (peek() != 'u') return false;
                    ++s_;
                    unsigned lo;
                    if (!hex4(lo) || lo < 0xDC00 || lo > 0xDFFF) return false;
                    cp = (((cp - 0xD800) << 10) | (lo - 0xDC00)) + 0x10000;
                }
                put_utf8(o, cp);
                break;
            }
            default: return false;
            }
        }
    }
    bool array(Value &v, int depth) {
        v.kind = Kind::Array;
        ++s_;
        ws();
        if (peek() == ']') { ++s_; return true; }
        for (;;) {
            v.items.emplace_back();
            if (!value(v.items.back(), depth + 1)) return false;
            ws();
            if (peek() == ',') { ++s_; ws(); continue; }
            if (peek() == ']') { ++s_; return true; }
            return false;
        }
    }
    bool object(Value &v, int depth) {
        v.kind = Kind::Object;
        ++s_;
        ws();
        if (peek() == '}') { ++s_; return true; }
        for (;;) {
            if (peek() != '"') return false;
            std::string key;
            if (!string(key)) return false;
            ws();
            if (peek() != ':') return false;
            ++s_;
            ws();
            v.members.emplace_back(std::move(key), Value());
            if (!value(v.members.back().second, depth + 1)) return false;
            ws();
            if (peek() == ',') { ++s_; ws(); continue; }
            if (peek() == '}') { ++s_; return true; }
            return false;
        }
    }

    static bool digit(char c) { return c >= '0' && c <= '9'; }

    /* exactly-rounded 10^n, n in [0, 308] (rapidjson internal/pow10.h holds the
     * same values as double literals) */
    static double pow10(int n) {
        static double table[309];
        static bool ready = false;
        if (!ready) {
            char buf[16];
            for (int i = 0; i <= 308; ++i) {
                std::snprintf(buf, sizeof buf, "1e%d", i);
                table[i] = std::strtod(buf, nullptr);
            }
            ready = true;
        }
        return table[n];
    }
    static double fast_path(double significand, int exp) {        /* internal/strtod.h */
        if (exp < -308) return 0.0;
        if (exp >= 0) return significand * pow10(exp);
        return significand / pow10(-exp);
    }
    static double normal_precision(double d, int p) {
        if (p < -308) {
            d = fast_path(d, -308);
            d = fast_path(d, p + 308);
        } else {
            d = fast_path(d, p);
        }
        return d;
    }

    /* rapidjson reader.h ParseNumber, default flags, 64-bit build. */
    bool number(Value &v) {
        bool minus = false;
        if (peek() == '-') { minus = true; ++s_; }
        unsigned i = 0;
        uint64_t i64 = 0;
        bool use64 = false;
        int sig = 0;
        if (peek() == '0') {
            i = 0;
            ++s_;
        } else if (peek() >= '1' && peek() <= '9') {
            i = (unsigned)(*s_++ - '0');
            if (minus) {
                while (digit(peek())) {
                    if (i >= 214748364u) {
                        if (i != 214748364u || peek() > '8') { i64 = i; use64 = true; break; }
                    }
                    i = i * 10 + (unsigned)(*s_++ - '0');
                    ++sig;
                }
            } else {
                while (digit(peek())) {
                    if (i >= 429496729u) {
                        if (i != 429496729u || peek() > '5') { i64 = i; use64 = true; break; }
                    }
                    i = i * 10 + (unsigned)(*s_++ - '0');
                    ++sig;
                }
            }
        } else {
            return false;
        }

        bool use_double = false;
        double d = 0.0;
        if (use64) {
            if (minus) {
                while (digit(peek())) {
                    if (i64 >= 0x0CCCCCCCCCCCCCCCull) {
                        if (i64 != 0x0CCCCCCCCCCCCCCCull || peek() > '8') {
                            d = (double)i64; use_double = true; break;
                        }
                    }
                    i64 = i64 * 10 + (unsigned)(*s_++ - '0');
                    ++sig;
                }
            } else {
                while (digit(peek())) {
                    if (i64 >= 0x1999999999999999ull) {
                        if (i64 != 0x1999999999999999ull || peek() > '5') {
                            d = (double)i64; use_double = true; break;
                        }
                    }
                    i64 = i64 * 10 + (unsigned)(*s_++ - '0');
                    ++sig;
                }
            }
        }
        if (use_double)
            while (digit(peek())) d = d * 10 + (*s_++ - '0');

        int exp_frac = 0;
        if (peek() == '.') {
            ++s_;
            if (!digit(peek())) return false;
            if (!use_double) {
                if (!use64) i64 = i;
                while (digit(peek())) {
                    if (i64 > 0x1FFFFFFFFFFFFFull) break;
                    i64 = i64 * 10 + (unsigned)(*s_++ - '0');
                    --exp_frac;
                    if (i64 != 0) ++sig;
                }
                d = (double)i64;
                use_double = true;
            }
            while (digit(peek())) {
                if (sig < 17) {
                    d = d * 10.0 + (*s_++ - '0');
                    --exp_frac;
                    if (d > 0.0) ++sig;
                } else {
                    ++s_;
                }
            }
        }

        int exp = 0;
        if (peek() == 'e' || peek() == 'E') {
            ++s_;
            if (!use_double) { d = (double)(use64 ? i64 : i); use_double = true; }
            bool exp_minus = false;
            if (peek() == '+') ++s_;
            else if (peek() == '-') { exp_minus = true; ++s_; }
            if (!digit(peek())) return false;
            exp = *s_++ - '0';
            if (exp_minus) {
                const int max_exp = (exp_frac + 2147483639) / 10;
                while (digit(peek())) {
                    exp = exp * 10 + (*s_++ - '0');
                    if (exp > max_exp) while (digit(peek())) ++s_;
                }
            } else {
                const int max_exp = 308 - exp_frac;
                while (digit(peek())) {
                    exp = exp * 10 + (*s_++ - '0');
                    if (exp > max_exp) return false;   /* kParseErrorNumberTooBig */
                }
            }
            if (exp_minus) exp = -exp;
        }

        if (use_double) {
            const int p = exp + exp_frac;
            d = normal_precision(d, p);
            if (d > std::numeric_limits<double>::max()) return false;
            v.num = minus ? -d : d;
            v.is_double = true;
            v.is_int = false;
        } else if (use64) {
            /* Int64 / Uint64: kIntFlag only when the value fits int32 (document.h) */
            if (minus) {
                const int64_t x = (int64_t)(~i64 + 1);
                v.num = (double)x;
                v.is_int = x >= std::numeric_limits<int32_t>::min() && x <= std::numeric_limits<int32_t>::max();
            } else {
                v.num = (double)i64;
                v.is_int = i64 <= (uint64_t)std::numeric_limits<int32_t>::max();
            }
        } else {
            if (minus) {
                const int32_t x = (int32_t)(~i + 1);
                v.num = (double)x;
                v.is_int = true;
            } else {
                v.num = (double)i;
                v.is_int = (i & 0x80000000u) == 0;
            }
        }
        return true;
    }
};

/* ---------------------------------------------------------------------- */
/*  crt_json.cpp restated over the DOM                                     */
/* ---------------------------------------------------------------------- */
static bool get_vector(const Value *v, crt_vec3 &out) {                   /* :34-43 */
    if (!v || !v->IsArray() || v->Size() != 3) return false;
    for (int k = 0; k < 3; ++k)
        if (!v->items[k].IsNumber()) return false;
    out.x = v->items[0].GetFloat();
    out.y = v->items[1].GetFloat();
    out.z = v->items[2].GetFloat();
    return true;
}

static bool get_matrix(const Value *v, float out[9]) {                     /* :45-61 */
    if (!v || !v->IsArray() || v->Size() != 9) return false;
    for (int k = 0; k < 9; ++k) {
        if (!v->items[k].IsNumber()) return false;
        out[k] = v->items[k].GetFloat();
    }
    return true;
}

static bool get_vector_array(const Value &v, std::vector<float> &out) {    /* :79-94 */
    if (!v.IsArray() || v.Size() % 3 != 0) return false;
    out.clear();
    out.reserve(v.Size());
    for (size_t i = 0; i < v.Size(); ++i) {
        if (!v.items[i].IsNumber()) return false;
        out.push_back(v.items[i].GetFloat());
    }
    return true;
}

static bool get_int_array(const Value &v, std::vector<int32_t> &out) {     /* :63-77 */
    if (!v.IsArray()) return false;
    out.clear();
    out.reserve(v.Size());
    for (const Value &x : v.items) {
        if (!x.IsInt()) return false;
        out.push_back(x.GetInt());
    }
    return true;
}

static bool parse_textures(const Value &v, SceneFile &sf, std::unordered_map<std::string, int32_t> &names,
                           const char *asset_root, std::string &why) {   /* :375-453 */
    if (!v.IsArray()) return false;
    for (size_t i = 0; i < v.Size(); ++i) {
        const Value &t = v.items[i];
        if (!t.IsObject()) return false;
        const Value *name = t.Find("name");
        if (!name || !name->IsString()) return false;
        names[name->str] = (int32_t)i;
        const Value *type = t.Find("type");
        if (!type) return false;
        crt_texture_desc d;
        std::memset(&d, 0, sizeof d);
        if (type->Equals("albedo")) {                                         /* :275-287 */
            d.type = CRT_TEXTURE_ALBEDO;
            if (!get_vector(t.Find("albedo"), d.color0)) return false;
        } else if (type->Equals("edges")) {                                   /* :289-317 */
            d.type = CRT_TEXTURE_EDGES;
            const Value *w = t.Find("edge_width");
            if (!w || !w->IsNumber()) return false;
            if (!get_vector(t.Find("edge_color"), d.color0)) return false;
            if (!get_vector(t.Find("inner_color"), d.color1)) return false;
            d.scalar = w->GetFloat();
        } else if (type->Equals("checker")) {                                 /* :319-347 */
            d.type = CRT_TEXTURE_CHECKER;
            const Value *a = t.Find("color_A"), *b = t.Find("color_B"), *sz = t.Find("square_size");
            if (!a || !b || !sz || !sz->IsNumber()) return false;
            if (!get_vector(a, d.color0) || !get_vector(b, d.color1)) return false;
            d.scalar = sz->GetFloat();
        } else if (type->Equals("bitmap")) {                                  /* :349-368 */
            const Value *fp = t.Find("file_path");
            if (!fp || !fp->IsString()) return false;
            /* asset_root / file_path.relative_path() (:358-360): the root name
             * and root directory are dropped, so "/textures/a.jpg" is read
             * under the scene's directory */
            std::string rel = fp->str;
            while (!rel.empty() && rel[0] == '/') rel.erase(0, 1);
            const std::string root = asset_root ? asset_root : "";
            const std::string path = root.empty() ? rel : (root.back() == '/' ? root + rel : root + "/" + rel);
            std::ifstream in(path, std::ios::in | std::ios::binary);
            std::vector<uint8_t> bytes;
            if (in.is_open()) bytes.assign(std::istreambuf_iterator<char>(in), std::istreambuf_iterator<char>());
            int bw = 0, bh = 0, comps = 0;
            std::vector<uint8_t> rgb;
            std::string dwhy;
            /* a failed read_stb drops the whole texture list (crt_json.cpp:582-588) */
            if (!in.is_open()) {
                why = "bitmap texture '" + fp->str + "': cannot open " + path;
                return false;
            }
            if (!decode_image_rgb8(bytes.data(), bytes.size(), bw, bh, comps, rgb, dwhy) || comps != 3) {
                why = "bitmap texture '" + fp->str + "': " + (dwhy.empty() ? "not 3 components" : dwhy);
                return false;
            }
            d.type = CRT_TEXTURE_BITMAP;
            d.bitmap_width = bw;
            d.bitmap_height = bh;
            std::vector<float> texels(rgb.size());
            for (size_t k = 0; k < rgb.size(); ++k) texels[k] = rgb[k] / 255.0f;   /* crt_image_stbi.cpp:29-37 */
            sf.bitmaps.resize(sf.textures.size() + 1);
            sf.bitmaps.back() = std::move(texels);
        } else {
            return false;
        }
        sf.textures.push_back(d);
    }
    return true;
}

static bool parse_materials(const Value &v, SceneFile &sf,
                            const std::unordered_map<std::string, int32_t> &names) {   /* :460-539 */
    if (!v.IsArray() || v.Size() == 0) return false;
    for (const Value &m : v.items) {
        if (!m.IsObject()) return false;
        const Value *type = m.Find("type");
        if (!type) return false;
        const Value *smooth = m.Find("smooth_shading");
        if (!smooth || !smooth->IsBool()) return false;
        bool cull = false;
        if (const Value *bf = m.Find("back_face_culling")) {
            if (!bf->IsBool()) return false;
            cull = bf->GetBool();
        }
        crt_material_desc d;
        std::memset(&d, 0, sizeof d);
        if (type->Equals("diffuse")) d.type = CRT_MATERIAL_DIFFUSE;
        else if (type->Equals("reflective")) d.type = CRT_MATERIAL_REFLECTIVE;
        else if (type->Equals("refractive")) d.type = CRT_MATERIAL_REFRACTIVE;
        else if (type->Equals("constant")) d.type = CRT_MATERIAL_CONSTANT;
        else return false;
        d.ior = 1.0f;
        d.albedo_texture_index = -1;
        if (d.type != CRT_MATERIAL_REFRACTIVE) {
            const Value *alb = m.Find("albedo");
            if (!alb) return false;
            if (alb->IsString()) {
                auto it = names.find(alb->str);
                if (it == names.end()) return false;
                d.albedo_texture_index = it->second;
            } else {
                crt_texture_desc t;
                std::memset(&t, 0, sizeof t);
                t.type = CRT_TEXTURE_ALBEDO;
                if (!get_vector(alb, t.color0)) return false;
                d.albedo_texture_index = (int32_t)sf.textures.size();
                sf.textures.push_back(t);
            }
        } else if (const Value *ior = m.Find("ior")) {
            if (!ior->IsNumber()) return false;
            d.ior = ior->GetFloat();
        }
        d.smooth_shading = smooth->GetBool() ? 1 : 0;
        d.back_face_culling = cull ? 1 : 0;
        sf.materials.push_back(d);
    }
    return true;
}

static bool parse_meshes(const Value &v, SceneFile &sf, std::string &why) {   /* :150-218 */
    if (!v.IsArray()) return false;
    for (const Value &o : v.items) {
        if (!o.IsObject()) return false;
        const Value *p = o.Find("vertices");
        if (!p || !p->IsArray()) return false;
        const Value *t = o.Find("triangles");
        if (!t || !t->IsArray()) return false;
        if (t->Size() % 3 != 0) return false;
    }
    for (const Value &o : v.items) {
        const Value *mi = o.Find("material_index");
        if (!mi || !mi->IsInt()) return false;
        SceneFile::Mesh mesh;
        mesh.material_index = mi->GetInt();
        if (!get_vector_array(*o.Find("vertices"), mesh.positions)) return false;
        if (!get_int_array(*o.Find("triangles"), mesh.indices)) return false;
        if (const Value *uv = o.Find("uvs")) {
            if (!get_vector_array(*uv, mesh.uvs)) return false;
            if (mesh.uvs.size() != mesh.positions.size()) return false;
            mesh.has_uvs = true;
        }
        /* UB in reference: material_triangle_flags[material_index] and the
         * vertex indices are not range-checked (crt_json.cpp:211-213,
         * crt_mesh.cpp:19).  Rejected here instead of reading out of bounds. */
        if (mesh.material_index < 0 || mesh.material_index >= (int32_t)sf.materials.size()) {
            why = "object material_index out of range";
            return false;
        }
        const int64_t nv = (int64_t)mesh.positions.size() / 3;
        for (int32_t ix : mesh.indices)
            if (ix < 0 || ix >= nv) { why = "triangle vertex index out of range"; return false; }
        sf.meshes_storage.push_back(std::move(mesh));
    }
    return true;
}

static bool parse_lights(const Value &v, SceneFile &sf) {                  /* :220-247 */
    if (!v.IsArray()) return false;
    for (const Value &l : v.items) {
        if (!l.IsObject()) return false;
        const Value *in = l.Find("intensity");
        if (!in || !in->IsNumber()) return false;
        crt_light_desc d;
        if (!get_vector(l.Find("position"), d.position)) return false;
        d.intensity = in->GetFloat();
        sf.lights.push_back(d);
    }
    return true;
}

static bool parse_scene(const Value &doc, SceneFile &sf, const char *asset_root, std::string &why) {   /* :541-647 */
    if (!doc.IsObject()) return false;
    const Value *settings = doc.Find("settings");
    if (!settings || !settings->IsObject()) return false;
    /* The reference compares against doc.MemberEnd() here (:555), so a missing
     * key is not caught and the end iterator is dereferenced (UB in reference);
     * treated as a parse failure. */
    if (!get_vector(settings->Find("background_color"), sf.desc.background_color)) return false;
    const Value *camera = doc.Find("camera");
    if (!camera) return false;
    const Value *img = settings->Find("image_settings");
    if (!img || !img->IsObject()) return false;   /* asserted object in reference (:120) */
    {                                                                        /* :119-143 */
        const Value *w = img->Find("width");
        if (!w || !w->IsInt()) return false;
        const Value *h = img->Find("height");
        if (!h || !h->IsInt()) return false;
        if (!camera->IsObject()) return false;                               /* :96-117 */
        if (!get_vector(camera->Find("position"), sf.desc.camera.location)) return false;
        if (!get_matrix(camera->Find("matrix"), sf.desc.camera.rotation)) return false;
        sf.desc.camera.fov_degrees = 90.0f;                                  /* crt_camera.h:13-15 */
        if (const Value *fov = camera->Find("fov_degrees")) {
            if (!fov->IsNumber()) return false;
            sf.desc.camera.fov_degrees = fov->GetFloat();
        }
        sf.desc.camera.width = w->GetInt();
        sf.desc.camera.height = h->GetInt();
    }
    sf.desc.bucket_size = 24;                                                /* crt_scene.h:16 */
    if (const Value *b = img->Find("bucket_size")) {
        if (!b->IsInt()) return false;
        sf.desc.bucket_size = b->GetInt();
    }
    std::unordered_map<std::string, int32_t> names;
    if (const Value *tx = doc.Find("textures")) {                            /* :582-588 */
        std::string tex_why;
        if (!parse_textures(*tx, sf, names, asset_root, tex_why)) {
            sf.textures.clear();
            sf.bitmaps.clear();
            names.clear();
            sf.warning = tex_why.empty() ? "texture list rejected" : tex_why;
        }
    }
    const Value *mats = doc.Find("materials");
    if (!mats) return false;
    if (!parse_materials(*mats, sf, names)) {
        if (!sf.warning.empty()) why = sf.warning;
        return false;
    }
    const Value *objs = doc.Find("objects");
    if (!objs) return false;
    if (!parse_meshes(*objs, sf, why)) return false;
    const Value *lights = doc.Find("lights");
    if (!lights) return false;
    if (!parse_lights(*lights, sf)) return false;
    sf.desc.gi_on = 0;
    sf.desc.reflections_on = 1;
    sf.desc.refractions_on = 1;
    if (const Value *g = settings->Find("gi_on")) {
        if (!g->IsBool()) return false;
        sf.desc.gi_on = g->GetBool();
    }
    if (const Value *r = settings->Find("reflections_on")) {
        if (!r->IsBool()) return false;
        sf.desc.reflections_on = r->GetBool();
    }
    if (const Value *r = settings->Find("refractions_on")) {
        if (!r->IsBool()) return false;
        sf.desc.refractions_on = r->GetBool();
    }
    return true;
}

}  // namespace json

void SceneFile::relink() {
    meshes.clear();
    for (const Mesh &m : meshes_storage) {
        crt_mesh_desc d;
        d.positions = m.positions.data();
        d.uvs = m.has_uvs ? m.uvs.data() : nullptr;
        d.vertex_count = (int64_t)m.positions.size() / 3;
        d.indices = m.indices.data();
        d.index_count = (int64_t)m.indices.size();
        d.material_index = m.material_index;
        meshes.push_back(d);
    }
    desc.meshes = meshes.data();
    desc.mesh_count = (int32_t)meshes.size();
    desc.materials = materials.data();
    desc.material_count = (int32_t)materials.size();
    bitmaps.resize(textures.size());
    for (size_t i = 0; i < textures.size(); ++i)
        textures[i].bitmap_rgb = bitmaps[i].empty() ? nullptr : bitmaps[i].data();
    desc.textures = textures.data();
    desc.texture_count = (int32_t)textures.size();
    desc.lights = lights.data();
    desc.light_count = (int32_t)lights.size();
}

int parse_scene_json(const char *text, size_t len, const char *asset_root, SceneFile &out) {
    json::Value doc;
    json::Parser p(text, len);
    if (!p.parse_document(doc)) return set_error(CRT_E_PARSE, "Could not parse JSON (syntax)");
    std::memset(&out.desc, 0, sizeof out.desc);
    std::string why;
    if (!json::parse_scene(doc, out, asset_root, why))
        return set_error(CRT_E_PARSE, why.empty() ? "Invalid CRT scene" : "Invalid CRT scene: " + why);
    out.relink();
    return CRT_OK;
}

}  // namespace crt_amd

using namespace crt_amd;

extern "C" {

int crt_scene_file_parse(const char *json_text, size_t len, const char *asset_root, crt_scene_file **out) {
    if (!json_text || !out) return set_error(CRT_E_INVALID, "null argument");
    *out = nullptr;
    std::unique_ptr<SceneFile> sf(new SceneFile());
    const int rc = parse_scene_json(json_text, len, asset_root, *sf);
    if (rc != CRT_OK) return rc;
    *out = reinterpret_cast<crt_scene_file *>(sf.release());
    return CRT_OK;
}

int crt_scene_file_load(const char *path, crt_scene_file **out) {
    if (!path || !out) return set_error(CRT_E_INVALID, "null argument");
    *out = nullptr;
    std::ifstream in(path, std::ios::in | std::ios::binary);
    if (!in.is_open()) return set_error(CRT_E_IO, std::string("Could not open input file: ") + path);
    std::stringstream ss;
    ss << in.rdbuf();
    const std::string text = ss.str();
    std::string root = path;
    const size_t slash = root.find_last_of('/');
    root = slash == std::string::npos ? std::string() : root.substr(0, slash);
    return crt_scene_file_parse(text.data(), text.size(), root.c_str(), out);
}

const crt_scene_desc *crt_scene_file_desc(const crt_scene_file *f) {
    return f ? &reinterpret_cast<const SceneFile *>(f)->desc : nullptr;
}

int crt_scene_file_set_resolution(crt_scene_file *f, int32_t width, int32_t height) {
    if (!f || width <= 0 || height <= 0) return set_error(CRT_E_INVALID, "bad resolution");
    SceneFile *sf = reinterpret_cast<SceneFile *>(f);
    sf->desc.camera.width = width;
    sf->desc.camera.height = height;
    return CRT_OK;
}

void crt_scene_file_destroy(crt_scene_file *f) { delete reinterpret_cast<SceneFile *>(f); }

}  // extern "C"
