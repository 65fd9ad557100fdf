// ply.cpp -- PLY point-cloud reader and writer (include/gsr_ply.h), host code.
//
// Replaces the `plyfile` calls of scene/gaussian_model.py:303-376 and
// scene/dataset_readers.py:120-143.  The body is moved in large blocks (fread / fwrite of
// up to 64 MiB at a time) and converted column-wise, so a 1M-Gaussian scene (248 MB) reads
// and writes at storage speed rather than plyfile's per-element Python overheads.
#include <cctype>
#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <memory>
#include <string>
#include <vector>

#include "../../include/gsr.h"
#include "../../include/gsr_ply.h"

namespace gsr {
int set_error(int code, const char* fmt, ...);  // api.hip
}

namespace {

enum Fmt { kAscii, kLittle, kBig };

struct Prop {
    std::string name;
    int type = 0;        // bytes of the scalar (1, 2, 4, 8)
    char kind = 'f';     // 'i' signed int, 'u' unsigned int, 'f' float
    bool list = false;   // list property: count type in (ctype, ckind), items in (type, kind)
    int ctype = 0;
    char ckind = 'u';
};

struct Element {
    std::string name;
    long long count = 0;
    std::vector<Prop> props;
    bool fixed() const {
        for (const Prop& p : props)
            if (p.list) return false;
        return true;
    }
    size_t row_bytes() const {
        size_t b = 0;
        for (const Prop& p : props) b += p.type;
        return b;
    }
};

bool parse_type(const std::string& t, int* bytes, char* kind) {
    static const struct { const char* n; int b; char k; } tab[] = {
        {"char", 1, 'i'},   {"int8", 1, 'i'},    {"uchar", 1, 'u'},  {"uint8", 1, 'u'},   {"short", 2, 'i'},
        {"int16", 2, 'i'},  {"ushort", 2, 'u'},  {"uint16", 2, 'u'}, {"int", 4, 'i'},     {"int32", 4, 'i'},
        {"uint", 4, 'u'},   {"uint32", 4, 'u'},  {"float", 4, 'f'},  {"float32", 4, 'f'}, {"double", 8, 'f'},
        {"float64", 8, 'f'}};
    for (const auto& e : tab)
        if (t == e.n) {
            *bytes = e.b;
            *kind = e.k;
            return true;
        }
    return false;
}

double decode(const unsigned char* p, int bytes, char kind, bool swap) {
    unsigned char b[8];
    for (int i = 0; i < bytes; i++) b[i] = swap ? p[bytes - 1 - i] : p[i];
    switch (bytes) {
        case 1: return kind == 'i' ? (double)(int8_t)b[0] : (double)b[0];
        case 2: {
            uint16_t v;
            memcpy(&v, b, 2);
            return kind == 'i' ? (double)(int16_t)v : (double)v;
        }
        case 4: {
            if (kind == 'f') {
                float f;
                memcpy(&f, b, 4);
                return f;
            }
            uint32_t v;
            memcpy(&v, b, 4);
            return kind == 'i' ? (double)(int32_t)v : (double)v;
        }
        default: {
            double d;
            memcpy(&d, b, 8);
            return d;
        }
    }
}

struct FileCloser {
    void operator()(FILE* f) const {
        if (f) fclose(f);
    }
};

}  // namespace

struct gsr_ply {
    std::string path;
    Fmt fmt = kLittle;
    std::vector<Element> elems;
    int vertex = -1;        // index of the vertex element
    long long body = 0;     // file offset of the first body byte
};

namespace {

int fail(const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    return gsr::set_error(GSR_ERR_ARGUMENT, "%s", buf);
}

}  // namespace

extern "C" int gsr_ply_open(const char* path, gsr_ply** out) {
    if (!path || !out) return fail("ply_open: null argument");
    *out = nullptr;
    std::unique_ptr<FILE, FileCloser> f(fopen(path, "rb"));
    if (!f) return fail("ply_open: cannot open %s", path);
    auto ply = std::make_unique<gsr_ply>();
    ply->path = path;
    char line[4096];
    int ln = 0;
    bool have_format = false;
    while (fgets(line, sizeof(line), f.get())) {
        ln++;
        std::string s(line);
        while (!s.empty() && (s.back() == '\n' || s.back() == '\r')) s.pop_back();
        if (ln == 1) {
            if (s != "ply") return fail("ply_open: %s is not a PLY file (first line '%s')", path, s.c_str());
            continue;
        }
        std::vector<std::string> tok;
        {
            size_t i = 0;
            while (i < s.size()) {
                while (i < s.size() && isspace((unsigned char)s[i])) i++;
                size_t j = i;
                while (j < s.size() && !isspace((unsigned char)s[j])) j++;
                if (j > i) tok.push_back(s.substr(i, j - i));
                i = j;
            }
        }
        if (tok.empty() || tok[0] == "comment" || tok[0] == "obj_info") continue;
        if (tok[0] == "end_header") {
            ply->body = ftell(f.get());
            break;
        }
        if (tok[0] == "format") {
            if (tok.size() < 2) return fail("ply_open: bad format line");
            if (tok[1] == "ascii") ply->fmt = kAscii;
            else if (tok[1] == "binary_little_endian") ply->fmt = kLittle;
            else if (tok[1] == "binary_big_endian") ply->fmt = kBig;
            else return fail("ply_open: unknown format '%s'", tok[1].c_str());
            have_format = true;
        } else if (tok[0] == "element") {
            if (tok.size() < 3) return fail("ply_open: bad element line");
            Element e;
            e.name = tok[1];
            e.count = atoll(tok[2].c_str());
            if (e.count < 0) return fail("ply_open: negative element count");
            ply->elems.push_back(e);
        } else if (tok[0] == "property") {
            if (ply->elems.empty()) return fail("ply_open: property before any element");
            Prop p;
            if (tok.size() >= 5 && tok[1] == "list") {
                p.list = true;
                if (!parse_type(tok[2], &p.ctype, &p.ckind) || !parse_type(tok[3], &p.type, &p.kind))
                    return fail("ply_open: bad list property types");
                p.name = tok[4];
            } else if (tok.size() >= 3) {
                if (!parse_type(tok[1], &p.type, &p.kind)) return fail("ply_open: unknown type '%s'", tok[1].c_str());
                p.name = tok[2];
            } else {
                return fail("ply_open: bad property line");
            }
            ply->elems.back().props.push_back(p);
        } else {
            return fail("ply_open: unexpected header line '%s'", s.c_str());
        }
    }
    if (!have_format || ply->body == 0) return fail("ply_open: %s: incomplete header", path);
    for (size_t i = 0; i < ply->elems.size(); i++)
        if (ply->elems[i].name == "vertex") ply->vertex = (int)i;
    if (ply->vertex < 0) return fail("ply_open: %s has no vertex element", path);
    *out = ply.release();
    return GSR_OK;
}

extern "C" void gsr_ply_close(gsr_ply* ply) { delete ply; }

extern "C" long long gsr_ply_vertex_count(const gsr_ply* ply) {
    return ply ? ply->elems[ply->vertex].count : -1;
}

extern "C" int gsr_ply_property_count(const gsr_ply* ply) {
    return ply ? (int)ply->elems[ply->vertex].props.size() : -1;
}

extern "C" const char* gsr_ply_property_name(const gsr_ply* ply, int i) {
    if (!ply || i < 0 || i >= (int)ply->elems[ply->vertex].props.size()) return nullptr;
    return ply->elems[ply->vertex].props[i].name.c_str();
}

namespace {

// store one value of column k, row v: as float32, or in the property's own type (raw)
struct Sink {
    void* const* out;
    const long long* stride;
    bool raw;
    void from_bytes(int k, long long v, const unsigned char* p, int bytes, char kind, bool swap) const {
        char* dst = (char*)out[k] + v * stride[k];
        if (!raw) {
            const float x = (float)decode(p, bytes, kind, swap);
            memcpy(dst, &x, 4);
        } else if (!swap) {
            memcpy(dst, p, bytes);
        } else {
            for (int i = 0; i < bytes; i++) dst[i] = (char)p[bytes - 1 - i];
        }
    }
    void from_double(int k, long long v, double x, int bytes, char kind) const {
        char* dst = (char*)out[k] + v * stride[k];
        if (!raw) {
            const float f = (float)x;
            memcpy(dst, &f, 4);
            return;
        }
        switch (kind == 'f' ? bytes * 10 : kind == 'i' ? bytes : bytes + 100) {
            case 40: { const float f = (float)x; memcpy(dst, &f, 4); break; }
            case 80: memcpy(dst, &x, 8); break;
            case 1: { const int8_t t = (int8_t)x; memcpy(dst, &t, 1); break; }
            case 2: { const int16_t t = (int16_t)x; memcpy(dst, &t, 2); break; }
            case 4: { const int32_t t = (int32_t)x; memcpy(dst, &t, 4); break; }
            case 101: { const uint8_t t = (uint8_t)x; memcpy(dst, &t, 1); break; }
            case 102: { const uint16_t t = (uint16_t)x; memcpy(dst, &t, 2); break; }
            default: { const uint32_t t = (uint32_t)x; memcpy(dst, &t, 4); break; }
        }
    }
};

int read_impl(gsr_ply* ply, int n, const char* const* names, const Sink& sink) {
    const Element& V = ply->elems[ply->vertex];
    std::vector<int> col(n);
    std::vector<size_t> coff(n, 0);
    for (int k = 0; k < n; k++) {
        col[k] = -1;
        size_t o = 0;
        for (size_t j = 0; j < V.props.size(); j++) {
            if (V.props[j].name == names[k]) {
                col[k] = (int)j;
                coff[k] = o;
            }
            o += V.props[j].type;
        }
        if (col[k] < 0) return fail("ply_read: %s has no vertex property '%s'", ply->path.c_str(), names[k]);
        if (V.props[col[k]].list) return fail("ply_read: vertex property '%s' is a list", names[k]);
    }
    std::unique_ptr<FILE, FileCloser> f(fopen(ply->path.c_str(), "rb"));
    if (!f || fseek(f.get(), ply->body, SEEK_SET) != 0) return fail("ply_read: cannot reopen %s", ply->path.c_str());
    const long long N = V.count;

    if (ply->fmt == kAscii) {
        std::string line;
        auto next_line = [&]() -> bool {
            line.clear();
            int c;
            while ((c = fgetc(f.get())) != EOF && c != '\n') line.push_back((char)c);
            return !(c == EOF && line.empty());
        };
        for (int e = 0; e < ply->vertex; e++)  // the elements before the vertex one: a line per row
            for (long long r = 0; r < ply->elems[e].count; r++)
                if (!next_line()) return fail("ply_read: truncated ascii body");
        std::vector<double> vals(V.props.size());
        for (long long v = 0; v < N; v++) {
            if (!next_line()) return fail("ply_read: truncated ascii body at vertex %lld", v);
            const char* p = line.c_str();
            for (size_t j = 0; j < V.props.size(); j++) {
                char* end = nullptr;
                vals[j] = strtod(p, &end);
                if (end == p) return fail("ply_read: bad ascii value at vertex %lld", v);
                p = end;
            }
            for (int k = 0; k < n; k++) {
                const Prop& pr = V.props[col[k]];
                sink.from_double(k, v, vals[col[k]], pr.type, pr.kind);
            }
        }
        return GSR_OK;
    }

    const bool swap = ply->fmt == kBig;
    // skip the elements before the vertex one
    for (int e = 0; e < ply->vertex; e++) {
        const Element& E = ply->elems[e];
        if (E.fixed()) {
            if (fseek(f.get(), (long)(E.count * (long long)E.row_bytes()), SEEK_CUR) != 0)
                return fail("ply_read: truncated body");
            continue;
        }
        for (long long r = 0; r < E.count; r++) {  // rows with lists: read the counts as we go
            for (const Prop& p : E.props) {
                unsigned char tmp[8];
                if (!p.list) {
                    if (fread(tmp, 1, p.type, f.get()) != (size_t)p.type) return fail("ply_read: truncated body");
                    continue;
                }
                if (fread(tmp, 1, p.ctype, f.get()) != (size_t)p.ctype) return fail("ply_read: truncated body");
                const long long c = (long long)decode(tmp, p.ctype, p.ckind, swap);
                if (fseek(f.get(), (long)(c * p.type), SEEK_CUR) != 0) return fail("ply_read: truncated body");
            }
        }
    }
    if (!V.fixed()) {  // a vertex element with list properties: row by row
        std::vector<unsigned char> row;
        std::vector<size_t> poff(V.props.size());
        for (long long v = 0; v < N; v++) {
            row.clear();
            size_t off = 0;
            for (size_t j = 0; j < V.props.size(); j++) {
                const Prop& p = V.props[j];
                poff[j] = off;
                unsigned char tmp[8];
                if (!p.list) {
                    if (fread(tmp, 1, p.type, f.get()) != (size_t)p.type) return fail("ply_read: truncated body");
                    row.insert(row.end(), tmp, tmp + p.type);
                    off += p.type;
                } else {
                    if (fread(tmp, 1, p.ctype, f.get()) != (size_t)p.ctype) return fail("ply_read: truncated body");
                    const long long c = (long long)decode(tmp, p.ctype, p.ckind, swap);
                    if (fseek(f.get(), (long)(c * p.type), SEEK_CUR) != 0) return fail("ply_read: truncated body");
                    row.insert(row.end(), tmp, tmp + p.ctype);
                    off += p.ctype;
                }
            }
            for (int k = 0; k < n; k++) {
                const Prop& p = V.props[col[k]];
                sink.from_bytes(k, v, row.data() + poff[col[k]], p.type, p.kind, swap);
            }
        }
        return GSR_OK;
    }
    const size_t rb = V.row_bytes();
    const long long rows_per_block = rb ? std::max<long long>(1, (64ll << 20) / (long long)rb) : N;
    std::vector<unsigned char> buf((size_t)std::min<long long>(N, rows_per_block) * rb + 1);
    for (long long v0 = 0; v0 < N; v0 += rows_per_block) {
        const long long nr = std::min(rows_per_block, N - v0);
        if (fread(buf.data(), rb, (size_t)nr, f.get()) != (size_t)nr)
            return fail("ply_read: %s: truncated body (%lld of %lld vertices)", ply->path.c_str(), v0, N);
        for (int k = 0; k < n; k++) {
            const Prop& p = V.props[col[k]];
            const unsigned char* src = buf.data() + coff[k];
            const long long st = sink.stride[k];
            char* dst = (char*)sink.out[k] + v0 * st;
            if (!swap && p.type == 4 && (sink.raw || p.kind == 'f')) {  // float32 / any 4-byte raw: moves
                for (long long r = 0; r < nr; r++) memcpy(dst + r * st, src + (size_t)r * rb, 4);
            } else {
                for (long long r = 0; r < nr; r++) sink.from_bytes(k, v0 + r, src + (size_t)r * rb, p.type, p.kind, swap);
            }
        }
    }
    return GSR_OK;
}

}  // namespace

extern "C" int gsr_ply_read_float(gsr_ply* ply, int n, const char* const* names, float* const* out,
                                  const long long* out_stride) {
    if (!ply || n < 0 || (n > 0 && (!names || !out || !out_stride))) return fail("ply_read: null argument");
    return read_impl(ply, n, names, Sink{(void* const*)out, out_stride, false});
}

extern "C" int gsr_ply_read_raw(gsr_ply* ply, int n, const char* const* names, void* const* out,
                                const long long* out_stride) {
    if (!ply || n < 0 || (n > 0 && (!names || !out || !out_stride))) return fail("ply_read: null argument");
    return read_impl(ply, n, names, Sink{out, out_stride, true});
}

extern "C" int gsr_ply_property_type(const gsr_ply* ply, int i, int* bytes, char* kind) {
    if (!ply || !bytes || !kind || i < 0 || i >= (int)ply->elems[ply->vertex].props.size())
        return fail("ply_property_type: bad argument");
    const Prop& p = ply->elems[ply->vertex].props[i];
    *bytes = p.type;
    *kind = p.list ? 'l' : p.kind;
    return GSR_OK;
}

extern "C" int gsr_ply_write(const char* path, long long N, int n, const char* const* names, const char* types,
                             const void* const* columns, const long long* strides) {
    if (!path || N < 0 || n <= 0 || !names || !types || (N > 0 && (!columns || !strides)))
        return fail("ply_write: bad argument");
    std::vector<int> bytes(n);
    size_t rb = 0;
    std::string header = "ply\nformat binary_little_endian 1.0\nelement vertex " + std::to_string(N) + "\n";
    // column type codes as Python's struct module spells them; header names as plyfile writes them
    static const struct { char code; int b; const char* name; } tab[] = {
        {'b', 1, "char"}, {'B', 1, "uchar"}, {'h', 2, "short"}, {'H', 2, "ushort"},
        {'i', 4, "int"},  {'I', 4, "uint"},  {'f', 4, "float"}, {'d', 8, "double"}};
    for (int k = 0; k < n; k++) {
        if (!names[k] || !names[k][0]) return fail("ply_write: empty property name");
        int b = 0;
        for (const auto& t : tab)
            if (t.code == types[k]) {
                b = t.b;
                header += std::string("property ") + t.name + " " + names[k] + "\n";
            }
        if (!b) return fail("ply_write: type '%c' of '%s' (one of bBhHiIfd)", types[k], names[k]);
        bytes[k] = b;
        rb += b;
    }
    header += "end_header\n";
    std::unique_ptr<FILE, FileCloser> f(fopen(path, "wb"));
    if (!f) return fail("ply_write: cannot create %s", path);
    if (fwrite(header.data(), 1, header.size(), f.get()) != header.size()) return fail("ply_write: write failed");
    const long long rows_per_block = std::max<long long>(1, (64ll << 20) / (long long)rb);
    std::vector<unsigned char> buf((size_t)std::min<long long>(std::max<long long>(N, 1), rows_per_block) * rb);
    for (long long v0 = 0; v0 < N; v0 += rows_per_block) {
        const long long nr = std::min(rows_per_block, N - v0);
        size_t off = 0;
        for (int k = 0; k < n; k++) {
            const char* src = (const char*)columns[k] + v0 * strides[k];
            unsigned char* dst = buf.data() + off;
            const long long st = strides[k];
            switch (bytes[k]) {  // constant-size copies: inlined moves, not library calls
                case 1: for (long long r = 0; r < nr; r++) dst[(size_t)r * rb] = (unsigned char)src[r * st]; break;
                case 2: for (long long r = 0; r < nr; r++) memcpy(dst + (size_t)r * rb, src + r * st, 2); break;
                case 4: for (long long r = 0; r < nr; r++) memcpy(dst + (size_t)r * rb, src + r * st, 4); break;
                default: for (long long r = 0; r < nr; r++) memcpy(dst + (size_t)r * rb, src + r * st, 8); break;
            }
            off += bytes[k];
        }
        if (fwrite(buf.data(), rb, (size_t)nr, f.get()) != (size_t)nr) return fail("ply_write: write failed");
    }
    if (fflush(f.get()) != 0) return fail("ply_write: write failed");
    return GSR_OK;
}
