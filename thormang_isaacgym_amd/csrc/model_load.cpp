// Native gym.load_asset for a URDF (tg_model_parse / tg_model_load, include/tgsim.h).
//
// The reference loads its assets through IsaacGym at run time
// (tasks/gogoro_new.py:198-213: gym.load_asset of scooter_V13.urdf, then the
// locked joints through the dof properties :257-262).  The Python host of this
// library does the same in model/urdf.py (parse, DFS link / DOF order, fixed and
// locked joints merged into rigid groups), abi.py (the tg_model_desc arrays and
// their hash) and model/codegen.py (the specialisation's constexpr traits,
// compiled by hipRTC through tg_model_jit).  This unit restates those three
// steps in C++, so a caller without Python (cgo, JNI, a C host) can load a URDF
// with one call; tests/test_model_load.py checks it against the Python path
// array for array and text for text.
//
// Conventions (model/urdf.py): bodies are the URDF links in depth-first order
// from the root link, children in joint-declaration order; DOFs are the
// non-fixed joints in that order; a joint frame equals its child-link frame at
// q = 0; continuous joints are revolute without limits; collision boxes and
// spheres are kept, a mesh collision becomes the torus fitted to its OBJ
// profile (tyres) when a mesh directory is given, other geometry is ignored.
// Arithmetic in double, arrays stored as float32, as the Python host does.
#include <stdint.h>

#include <algorithm>
#include <cctype>
#include <cerrno>
#include <clocale>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <functional>
#include <locale>
#include <map>
#include <set>
#include <sstream>
#include <string>
#include <vector>

#include "../../include/tgsim.h"

namespace {

// ------------------------------------------------------------------ XML
struct XNode {
    std::string tag;
    std::vector<std::pair<std::string, std::string>> attrs;
    std::vector<XNode> kids;
    const std::string *attr(const char *k) const {
        for (const auto &a : attrs)
            if (a.first == k) return &a.second;
        return nullptr;
    }
    const XNode *child(const char *t) const {
        for (const auto &c : kids)
            if (c.tag == t) return &c;
        return nullptr;
    }
};

std::string xml_unescape(const std::string &s) {
    std::string o;
    for (size_t i = 0; i < s.size(); ++i) {
        if (s[i] != '&') {
            o += s[i];
            continue;
        }
        const size_t e = s.find(';', i);
        if (e == std::string::npos) {
            o += s[i];
            continue;
        }
        const std::string n = s.substr(i + 1, e - i - 1);
        if (n == "amp") o += '&';
        else if (n == "lt") o += '<';
        else if (n == "gt") o += '>';
        else if (n == "quot") o += '"';
        else if (n == "apos") o += '\'';
        else if (!n.empty() && n[0] == '#') o += (char)std::strtol(n.c_str() + (n.size() > 1 && n[1] == 'x' ? 2 : 1), nullptr, n.size() > 1 && n[1] == 'x' ? 16 : 10);
        else o += "&" + n + ";";
        i = e;
    }
    return o;
}

// a minimal XML reader for URDF: elements, attributes, comments, processing
// instructions and DOCTYPE skipped, character data ignored
struct XmlReader {
    const std::string &s;
    size_t p = 0;
    std::string err;
    explicit XmlReader(const std::string &t) : s(t) {}
    void ws() {
        while (p < s.size() && std::isspace((unsigned char)s[p])) ++p;
    }
    bool skip_misc() {   // comments, <? ?>, <! >
        for (;;) {
            const size_t lt = s.find('<', p);
            if (lt == std::string::npos) return false;
            p = lt;
            if (s.compare(p, 4, "<!--") == 0) {
                const size_t e = s.find("-->", p + 4);
                if (e == std::string::npos) return false;
                p = e + 3;
            } else if (s.compare(p, 2, "<?") == 0) {
                const size_t e = s.find("?>", p + 2);
                if (e == std::string::npos) return false;
                p = e + 2;
            } else if (s.compare(p, 2, "<!") == 0) {
                const size_t e = s.find('>', p + 2);
                if (e == std::string::npos) return false;
                p = e + 1;
            } else {
                return true;
            }
        }
    }
    int depth = 0;
    static constexpr int kMaxDepth = 256;   // nesting bound: no stack exhaustion on hostile input
    bool element(XNode &n) {   // at '<' of a start tag
        if (++depth > kMaxDepth) return fail("elements nested deeper than " + std::to_string(kMaxDepth));
        ++p;
        const size_t b = p;
        while (p < s.size() && !std::isspace((unsigned char)s[p]) && s[p] != '>' && s[p] != '/') ++p;
        n.tag = s.substr(b, p - b);
        for (;;) {
            ws();
            if (p >= s.size()) return fail("unterminated tag <" + n.tag);
            if (s[p] == '/') {
                if (p + 1 >= s.size() || s[p + 1] != '>') return fail("bad tag end in <" + n.tag);
                p += 2;
                --depth;
                return true;
            }
            if (s[p] == '>') {
                ++p;
                break;
            }
            const size_t kb = p;
            while (p < s.size() && s[p] != '=' && !std::isspace((unsigned char)s[p])) ++p;
            const std::string key = s.substr(kb, p - kb);
            ws();
            if (p >= s.size() || s[p] != '=') return fail("attribute without value in <" + n.tag);
            ++p;
            ws();
            if (p >= s.size() || (s[p] != '"' && s[p] != '\'')) return fail("unquoted attribute in <" + n.tag);
            const char q = s[p++];
            const size_t e = s.find(q, p);
            if (e == std::string::npos) return fail("unterminated attribute in <" + n.tag);
            n.attrs.emplace_back(key, xml_unescape(s.substr(p, e - p)));
            p = e + 1;
        }
        for (;;) {   // content
            if (!skip_misc()) return fail("unterminated element <" + n.tag);
            if (s.compare(p, 2, "</") == 0) {
                const size_t e = s.find('>', p);
                if (e == std::string::npos) return fail("unterminated end tag");
                std::string t = s.substr(p + 2, e - p - 2);
                while (!t.empty() && std::isspace((unsigned char)t.back())) t.pop_back();
                if (t != n.tag) return fail("mismatched </" + t + "> for <" + n.tag + ">");
                p = e + 1;
                --depth;
                return true;
            }
            n.kids.emplace_back();
            if (!element(n.kids.back())) return false;
        }
    }
    bool fail(const std::string &m) {
        err = m;
        return false;
    }
    bool parse(XNode &root) {
        if (!skip_misc()) return fail("no root element");
        return element(root);
    }
};

// ------------------------------------------------------------------ model
enum { J_FIXED = 0, J_REV = 1, J_PRISM = 2 };
enum { S_TORUS = 0, S_BOX = 1, S_SPHERE = 2 };
typedef std::vector<double> V;

struct Link {
    std::string name;
    double mass = 0;
    double com[3] = {0, 0, 0}, inertia[6] = {0, 0, 0, 0, 0, 0};
    int parent = -1, joint = -1;
};
struct Joint {
    std::string name;
    int jtype = J_FIXED, parent = -1, child = -1, dof = -1;
    double pos[3] = {0, 0, 0}, rot[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1}, axis[3] = {1, 0, 0};
    double lower = -INFINITY, upper = INFINITY, effort = 0, velocity = 0;
    bool has_limits = false;
};
struct Shape {
    int kind = S_BOX, link = 0;
    double pos[3] = {0, 0, 0}, rot[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1}, params[4] = {0, 0, 0, 0};
    int np = 0;
    double friction = 1.0;
};

// one number token as the Python host's float() reads it (model/urdf.py):
// surrounding blanks allowed, decimal point '.' whatever LC_NUMERIC the host
// set (strtod_l in the "C" locale), "inf" / "infinity" / "nan" in any case
// with an optional sign, overflow to +-inf, underscores only between digits,
// and the WHOLE token consumed -- no hex floats (strtod's, not float()'s)
bool parse_float(const std::string &tok, double &out) {
    size_t b = tok.find_first_not_of(" \t\r\n"), e = tok.find_last_not_of(" \t\r\n");
    if (b == std::string::npos) return false;
    std::string t;
    for (size_t k = b; k <= e; ++k) {
        const char c = tok[k];
        if (c == 'x' || c == 'X' || c == '(') return false;   // no hex floats, no strtod "nan(n-char-seq)"
        if (c == '_') {   // float("1_000.5") == 1000.5; "1__0", "_1", "1_" are errors
            if (k == b || k == e || !std::isdigit((unsigned char)tok[k - 1]) || !std::isdigit((unsigned char)tok[k + 1]))
                return false;
            continue;
        }
        t += c;
    }
    static const locale_t c_loc = newlocale(LC_ALL_MASK, "C", (locale_t)0);
    if (c_loc == (locale_t)0) return false;   // no "C" locale object: report the value malformed, never UB
    char *end = nullptr;
    errno = 0;
    const double v = strtod_l(t.c_str(), &end, c_loc);
    if (end == t.c_str() || *end != '\0') return false;
    out = v;   // (ERANGE overflow: +-HUGE_VAL = +-inf, as float("1e999"); underflow: 0 or a denormal, as float())
    return true;
}

bool vec_attr(const XNode *el, const char *key, int n, double dflt, double *out, std::string &err) {
    for (int i = 0; i < n; ++i) out[i] = dflt;
    if (!el) return true;
    const std::string *v = el->attr(key);
    if (!v) return true;
    std::istringstream is(*v);
    std::string tok;
    int i = 0;
    for (; is >> tok; ++i)
        if (i >= n || !parse_float(tok, out[i])) break;
    if (i != n || (is >> tok)) {
        err = std::string("expected ") + std::to_string(n) + " numbers in " + key + "=\"" + *v + "\"";
        return false;
    }
    return true;
}

// one number attribute (absent: dflt), parsed as float() parses it
// (parse_float): a malformed value is an error, not a silent 0
bool num_attr(const XNode *el, const char *key, double dflt, double &out, std::string &err) {
    out = dflt;
    if (!el) return true;
    const std::string *v = el->attr(key);
    if (!v) return true;
    if (!parse_float(*v, out)) {
        err = std::string("malformed number in ") + el->tag + " " + key + "=\"" + *v + "\"";
        return false;
    }
    return true;
}

// URDF fixed-axis roll-pitch-yaw: R = Rz(y) Ry(p) Rx(r), row-major
void rpy_to_matrix(const double *rpy, double *R) {
    const double cr = std::cos(rpy[0]), sr = std::sin(rpy[0]), cp = std::cos(rpy[1]), sp = std::sin(rpy[1]),
                 cy = std::cos(rpy[2]), sy = std::sin(rpy[2]);
    const double m[9] = {cy * cp, cy * sp * sr - sy * cr, cy * sp * cr + sy * sr,
                         sy * cp, sy * sp * sr + cy * cr, sy * sp * cr - cy * sr,
                         -sp,     cp * sr,                cp * cr};
    std::memcpy(R, m, sizeof m);
}

void matmul3(const double *A, const double *B, double *C) {
    double t[9];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) t[3 * i + j] = A[3 * i] * B[j] + A[3 * i + 1] * B[3 + j] + A[3 * i + 2] * B[6 + j];
    std::memcpy(C, t, sizeof t);
}

// tyre torus fitted to an OBJ mesh (model/urdf.py fit_tire_torus): spin axis =
// the mesh axis of least extent; crown radius R + r, shoulder at |z| = 0.8 *
// half-width pins (R, r)
bool fit_tire_torus(const std::string &path, double scale, double &Rt, double &rt, int &ax, std::string &err) {
    std::ifstream f(path);
    if (!f) {
        err = "mesh " + path + " not found";
        return false;
    }
    std::vector<double> v;
    std::string line;
    while (std::getline(f, line)) {
        if (line.size() > 2 && line[0] == 'v' && line[1] == ' ') {
            std::istringstream is(line.substr(2));
            double x, y, z;
            if (is >> x >> y >> z) {
                v.push_back(x * scale);
                v.push_back(y * scale);
                v.push_back(z * scale);
            }
        }
    }
    const size_t n = v.size() / 3;
    if (n == 0) {
        err = "mesh " + path + " has no vertices";
        return false;
    }
    double lo[3], hi[3];
    for (int k = 0; k < 3; ++k) lo[k] = hi[k] = v[k];
    for (size_t i = 0; i < n; ++i)
        for (int k = 0; k < 3; ++k) {
            lo[k] = std::min(lo[k], v[3 * i + k]);
            hi[k] = std::max(hi[k], v[3 * i + k]);
        }
    double ext[3];
    for (int k = 0; k < 3; ++k) {
        const double c = (hi[k] + lo[k]) / 2;
        for (size_t i = 0; i < n; ++i) v[3 * i + k] -= c;
        ext[k] = (hi[k] - c) - (lo[k] - c);
    }
    ax = 0;
    for (int k = 1; k < 3; ++k)
        if (ext[k] < ext[ax]) ax = k;
    const int a1 = ax == 0 ? 1 : 0, a2 = ax == 2 ? 1 : 2;
    const double zs = 0.8 * ext[ax] / 2;
    double crown = -INFINITY, shoulder = -INFINITY;
    for (size_t i = 0; i < n; ++i) {
        const double z = v[3 * i + ax];
        const double rho = std::sqrt(v[3 * i + a1] * v[3 * i + a1] + v[3 * i + a2] * v[3 * i + a2]);
        if (std::fabs(z) < 0.05 * ext[ax]) crown = std::max(crown, rho);
        if (std::fabs(std::fabs(z) - zs) < 0.05 * ext[ax]) shoulder = std::max(shoulder, rho);
    }
    if (!std::isfinite(crown) || !std::isfinite(shoulder) || crown <= shoulder) {
        err = "mesh " + path + " is not a tyre profile (torus fit)";
        return false;
    }
    const double d = crown - shoulder;
    rt = (zs * zs + d * d) / (2 * d);
    Rt = crown - rt;
    return true;
}

}  // namespace

// the library-side model (opaque tg_model of include/tgsim.h)
struct tg_model {
    std::string name;
    std::vector<Link> links;
    std::vector<Joint> joints;
    std::vector<Shape> shapes;
    std::vector<std::string> dof_names;
    std::vector<int> dof_joint;
    std::vector<int> link_group, group_root, group_parent, group_dof, locked_dofs;
    // tg_model_desc arrays (float32 / int32, as abi.model_arrays)
    std::vector<int32_t> a_link_parent, a_link_group, a_link_dof, a_link_jtype, a_group_root, a_group_parent,
        a_dof_locked, a_shape_link, a_shape_kind;
    std::vector<float> a_link_origin, a_link_axis, a_link_inertia, a_shape_pose, a_shape_params, a_shape_friction;
    uint64_t hash = 0;
    std::string cname, source;
};

namespace {

// ------------------------------------------------------------------ SHA-1 (abi.model_hash)
struct Sha1 {
    uint32_t h[5] = {0x67452301u, 0xEFCDAB89u, 0x98BADCFEu, 0x10325476u, 0xC3D2E1F0u};
    unsigned char buf[64];
    uint64_t len = 0;
    size_t n = 0;
    static uint32_t rol(uint32_t x, int k) { return (x << k) | (x >> (32 - k)); }
    void block(const unsigned char *b) {
        uint32_t w[80];
        for (int i = 0; i < 16; ++i) w[i] = (uint32_t)b[4 * i] << 24 | (uint32_t)b[4 * i + 1] << 16 | (uint32_t)b[4 * i + 2] << 8 | b[4 * i + 3];
        for (int i = 16; i < 80; ++i) w[i] = rol(w[i - 3] ^ w[i - 8] ^ w[i - 14] ^ w[i - 16], 1);
        uint32_t a = h[0], bb = h[1], c = h[2], d = h[3], e = h[4];
        for (int i = 0; i < 80; ++i) {
            uint32_t f, k;
            if (i < 20) { f = (bb & c) | (~bb & d); k = 0x5A827999u; }
            else if (i < 40) { f = bb ^ c ^ d; k = 0x6ED9EBA1u; }
            else if (i < 60) { f = (bb & c) | (bb & d) | (c & d); k = 0x8F1BBCDCu; }
            else { f = bb ^ c ^ d; k = 0xCA62C1D6u; }
            const uint32_t t = rol(a, 5) + f + e + k + w[i];
            e = d; d = c; c = rol(bb, 30); bb = a; a = t;
        }
        h[0] += a; h[1] += bb; h[2] += c; h[3] += d; h[4] += e;
    }
    void update(const void *p, size_t m) {
        const unsigned char *b = (const unsigned char *)p;
        len += m;
        while (m > 0) {
            const size_t k = std::min(m, 64 - n);
            std::memcpy(buf + n, b, k);
            n += k; b += k; m -= k;
            if (n == 64) { block(buf); n = 0; }
        }
    }
    void digest(unsigned char out[20]) {
        const uint64_t bits = len * 8;
        const unsigned char pad = 0x80, zero = 0;
        update(&pad, 1);
        while (n != 56) update(&zero, 1);
        unsigned char lb[8];
        for (int i = 0; i < 8; ++i) lb[i] = (unsigned char)(bits >> (56 - 8 * i));
        update(lb, 8);
        for (int i = 0; i < 5; ++i)
            for (int k = 0; k < 4; ++k) out[4 * i + k] = (unsigned char)(h[i] >> (24 - 8 * k));
    }
};

// ------------------------------------------------------------------ build
bool build_model(const std::string &path, const std::string &name, const std::vector<std::string> &locked,
                 const std::string &mesh_root, tg_model &m, std::string &err) {
    std::ifstream f(path, std::ios::binary);
    if (!f) {
        err = "URDF " + path + " not found";
        return false;
    }
    std::stringstream ss;
    ss << f.rdbuf();
    const std::string text = ss.str();
    XNode robot;
    XmlReader rd(text);
    if (!rd.parse(robot)) {
        err = "URDF " + path + ": " + rd.err;
        return false;
    }
    std::map<std::string, const XNode *> link_el;
    std::vector<const XNode *> link_order, joint_el;
    for (const auto &c : robot.kids) {
        if (c.tag == "link" && c.attr("name")) {
            link_el[*c.attr("name")] = &c;
            link_order.push_back(&c);
        } else if (c.tag == "joint") {
            joint_el.push_back(&c);
        }
    }
    std::map<std::string, std::vector<const XNode *>> children;
    std::set<std::string> child_names;
    for (const XNode *j : joint_el) {
        const XNode *pa = j->child("parent"), *ch = j->child("child");
        if (!pa || !ch || !pa->attr("link") || !ch->attr("link") || !j->attr("name")) {
            err = "URDF " + path + ": joint without name / parent / child";
            return false;
        }
        children[*pa->attr("link")].push_back(j);
        if (!child_names.insert(*ch->attr("link")).second) {   // a tree: one parent joint per link
            err = "URDF " + path + ": link " + *ch->attr("link") + " is the child of more than one joint";
            return false;
        }
    }
    std::vector<std::string> roots;
    for (const XNode *l : link_order)
        if (!child_names.count(*l->attr("name"))) roots.push_back(*l->attr("name"));
    if (roots.size() != 1) {
        err = "URDF must have one root link, found " + std::to_string(roots.size());
        return false;
    }
    m.name = name;
    // depth-first, children in joint-declaration order (model/urdf.py load_urdf)
    std::function<int(const std::string &, int, int)> dfs;
    std::set<std::string> visited;
    bool ok = true;
    // the joint-tree depth is bounded like the XML nesting: a hostile chain of
    // links must not exhaust the stack through this recursion
    static constexpr int kMaxTreeDepth = 1024;
    int tdepth = 0;
    dfs = [&](const std::string &lname, int parent, int joint) -> int {
        if (tdepth >= kMaxTreeDepth) {
            err = "URDF: link chain deeper than " + std::to_string(kMaxTreeDepth);
            ok = false;
            return -1;
        }
        struct Depth {
            int &d;
            explicit Depth(int &x) : d(++x) {}
            ~Depth() { --d; }
        } depth_guard(tdepth);
        auto it = link_el.find(lname);
        if (it == link_el.end()) {
            err = "URDF: joint child link " + lname + " not declared";
            ok = false;
            return -1;
        }
        Link L;
        L.name = lname;
        L.parent = parent;
        L.joint = joint;
        if (!visited.insert(lname).second) {   // (unreachable with one parent per link; kept as the cycle guard)
            err = "URDF: link " + lname + " reached twice (joint cycle)";
            ok = false;
            return -1;
        }
        if (const XNode *in = it->second->child("inertial")) {
            const XNode *ms = in->child("mass");
            if (!num_attr(ms, "value", 0.0, L.mass, err)) {
                ok = false;
                return -1;
            }
            const XNode *o = in->child("origin");
            double rpy[3], R[9];
            if (!vec_attr(o, "xyz", 3, 0.0, L.com, err) || !vec_attr(o, "rpy", 3, 0.0, rpy, err)) {
                ok = false;
                return -1;
            }
            const XNode *ia = in->child("inertia");
            double ixx, ixy, ixz, iyy, iyz, izz;
            if (!num_attr(ia, "ixx", 0, ixx, err) || !num_attr(ia, "ixy", 0, ixy, err) ||
                !num_attr(ia, "ixz", 0, ixz, err) || !num_attr(ia, "iyy", 0, iyy, err) ||
                !num_attr(ia, "iyz", 0, iyz, err) || !num_attr(ia, "izz", 0, izz, err)) {
                ok = false;
                return -1;
            }
            const double I[9] = {ixx, ixy, ixz, ixy, iyy, iyz, ixz, iyz, izz};
            rpy_to_matrix(rpy, R);
            double RI[9], Rt[9], Iw[9];
            for (int i = 0; i < 3; ++i)
                for (int j = 0; j < 3; ++j) Rt[3 * i + j] = R[3 * j + i];
            matmul3(R, I, RI);
            matmul3(RI, Rt, Iw);
            const double in6[6] = {Iw[0], Iw[4], Iw[8], Iw[1], Iw[2], Iw[5]};
            std::memcpy(L.inertia, in6, sizeof in6);
        }
        m.links.push_back(L);
        const int li = (int)m.links.size() - 1;
        for (const XNode *j : children[lname]) {
            if (!ok) return -1;
            const std::string jt = j->attr("type") ? *j->attr("type") : "";
            Joint J;
            J.name = *j->attr("name");
            if (jt == "fixed") J.jtype = J_FIXED;
            else if (jt == "revolute" || jt == "continuous") J.jtype = J_REV;
            else if (jt == "prismatic") J.jtype = J_PRISM;
            else {
                err = "unsupported joint type " + jt + " (" + J.name + ")";
                ok = false;
                return -1;
            }
            J.parent = li;
            const XNode *o = j->child("origin");
            double rpy[3];
            if (!vec_attr(o, "xyz", 3, 0.0, J.pos, err) || !vec_attr(o, "rpy", 3, 0.0, rpy, err)) {
                ok = false;
                return -1;
            }
            rpy_to_matrix(rpy, J.rot);
            const XNode *a = j->child("axis");
            if (a) {
                if (!vec_attr(a, "xyz", 3, 0.0, J.axis, err)) {
                    ok = false;
                    return -1;
                }
            }
            double nrm = std::sqrt(J.axis[0] * J.axis[0] + J.axis[1] * J.axis[1] + J.axis[2] * J.axis[2]);
            if (nrm == 0.0) nrm = 1.0;
            for (int k = 0; k < 3; ++k) J.axis[k] /= nrm;
            if (const XNode *lim = j->child("limit")) {
                if (!num_attr(lim, "effort", 0.0, J.effort, err) || !num_attr(lim, "velocity", 0.0, J.velocity, err)) {
                    ok = false;
                    return -1;
                }
                if (jt != "continuous" && J.jtype != J_FIXED) {
                    if (!num_attr(lim, "lower", 0.0, J.lower, err) || !num_attr(lim, "upper", 0.0, J.upper, err)) {
                        ok = false;
                        return -1;
                    }
                    J.has_limits = true;
                }
            }
            if (J.jtype != J_FIXED) {
                J.dof = (int)m.dof_names.size();
                m.dof_names.push_back(J.name);
                m.dof_joint.push_back((int)m.joints.size());
            }
            m.joints.push_back(J);
            const int ji = (int)m.joints.size() - 1;
            const int ci = dfs(*j->child("child")->attr("link"), li, ji);
            if (!ok) return -1;
            m.joints[ji].child = ci;
        }
        return li;
    };
    dfs(roots[0], -1, -1);
    if (!ok) return false;
    // collision shapes, in link order
    for (size_t li = 0; li < m.links.size(); ++li) {
        for (const auto &c : link_el[m.links[li].name]->kids) {
            if (c.tag != "collision") continue;
            const XNode *geo = c.child("geometry");
            if (!geo || geo->kids.empty()) continue;
            const XNode &g = geo->kids[0];
            const XNode *o = c.child("origin");
            Shape S;
            S.link = (int)li;
            double rpy[3];
            if (!vec_attr(o, "xyz", 3, 0.0, S.pos, err) || !vec_attr(o, "rpy", 3, 0.0, rpy, err)) return false;
            rpy_to_matrix(rpy, S.rot);
            if (g.tag == "mesh" && !mesh_root.empty()) {
                std::string fn = g.attr("filename") ? *g.attr("filename") : "";
                fn = fn.substr(fn.find_last_of('/') + 1);
                double sc[3];
                if (!vec_attr(&g, "scale", 3, 1.0, sc, err)) return false;
                double Rt, rt;
                int ax;
                if (!fit_tire_torus(mesh_root + "/" + fn, sc[0], Rt, rt, ax, err)) return false;
                // the torus axis onto shape z: columns (ax+1, ax+2, ax) of I
                double Pa[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
                const int cols[3] = {(ax + 1) % 3, (ax + 2) % 3, ax};
                for (int k = 0; k < 3; ++k) Pa[3 * cols[k] + k] = 1.0;
                matmul3(S.rot, Pa, S.rot);
                S.kind = S_TORUS;
                S.params[0] = Rt;
                S.params[1] = rt;
                S.np = 2;
                m.shapes.push_back(S);
            } else if (g.tag == "box") {
                double sz[3];
                if (!vec_attr(&g, "size", 3, 0.0, sz, err)) return false;
                S.kind = S_BOX;
                for (int k = 0; k < 3; ++k) S.params[k] = sz[k] / 2;
                S.np = 3;
                m.shapes.push_back(S);
            } else if (g.tag == "sphere") {
                S.kind = S_SPHERE;
                if (!num_attr(&g, "radius", 0.0, S.params[0], err)) return false;
                S.np = 1;
                m.shapes.push_back(S);
            }
        }
    }
    // groups (model/urdf.py build_groups): a link starts a group at the root or
    // behind an active (non-fixed, non-locked) joint
    std::set<std::string> lk(locked.begin(), locked.end());
    for (const auto &n : lk)
        if (std::find(m.dof_names.begin(), m.dof_names.end(), n) == m.dof_names.end()) {
            err = "locked joint not in model: " + n;
            return false;
        }
    m.link_group.assign(m.links.size(), -1);
    for (size_t li = 0; li < m.links.size(); ++li) {
        const Link &L = m.links[li];
        bool starts = L.parent < 0;
        if (!starts) {
            const Joint &J = m.joints[L.joint];
            starts = J.jtype != J_FIXED && !lk.count(J.name);
        }
        if (starts) {
            const int g = (int)m.group_root.size();
            m.group_root.push_back((int)li);
            m.group_parent.push_back(L.parent < 0 ? -1 : m.link_group[L.parent]);
            m.group_dof.push_back(L.parent < 0 ? -1 : m.joints[L.joint].dof);
            m.link_group[li] = g;
        } else {
            m.link_group[li] = m.link_group[L.parent];
        }
    }
    for (size_t d = 0; d < m.dof_names.size(); ++d)
        if (lk.count(m.dof_names[d])) m.locked_dofs.push_back((int)d);
    return true;
}

// the tg_model_desc arrays and their hash (abi.model_arrays / model_hash)
void build_arrays(tg_model &m) {
    const size_t L = m.links.size(), D = m.dof_names.size(), S = m.shapes.size();
    m.a_link_parent.clear();
    for (const auto &l : m.links) {
        m.a_link_parent.push_back(l.parent);
        m.a_link_dof.push_back(l.joint >= 0 ? m.joints[l.joint].dof : -1);
        m.a_link_jtype.push_back(l.joint >= 0 ? m.joints[l.joint].jtype : J_FIXED);
        const double eye[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
        const double *R = l.joint >= 0 ? m.joints[l.joint].rot : eye;
        for (int k = 0; k < 9; ++k) m.a_link_origin.push_back((float)R[k]);
        for (int k = 0; k < 3; ++k) m.a_link_origin.push_back(l.joint >= 0 ? (float)m.joints[l.joint].pos[k] : 0.f);
        for (int k = 0; k < 3; ++k) m.a_link_axis.push_back(l.joint >= 0 ? (float)m.joints[l.joint].axis[k] : 0.f);
        m.a_link_inertia.push_back((float)l.mass);
        for (int k = 0; k < 3; ++k) m.a_link_inertia.push_back((float)l.com[k]);
        for (int k = 0; k < 6; ++k) m.a_link_inertia.push_back((float)l.inertia[k]);
    }
    m.a_link_group.assign(m.link_group.begin(), m.link_group.end());
    m.a_group_root.assign(m.group_root.begin(), m.group_root.end());
    m.a_group_parent.assign(m.group_parent.begin(), m.group_parent.end());
    m.a_dof_locked.assign(D, 0);
    for (int d : m.locked_dofs) m.a_dof_locked[d] = 1;
    for (const auto &s : m.shapes) {
        m.a_shape_link.push_back(s.link);
        m.a_shape_kind.push_back(s.kind);
        for (int k = 0; k < 9; ++k) m.a_shape_pose.push_back((float)s.rot[k]);
        for (int k = 0; k < 3; ++k) m.a_shape_pose.push_back((float)s.pos[k]);
        for (int k = 0; k < 4; ++k) m.a_shape_params.push_back(k < s.np ? (float)s.params[k] : 0.f);
        m.a_shape_friction.push_back((float)s.friction);
    }
    (void)L; (void)S;
    // sha1 over (key, bytes) in sorted key order, the first 8 digest bytes little-endian
    Sha1 h;
    auto put = [&](const char *k, const void *p, size_t n) {
        h.update(k, std::strlen(k));
        if (n) h.update(p, n);
    };
    put("dof_locked", m.a_dof_locked.data(), m.a_dof_locked.size() * 4);
    put("group_parent", m.a_group_parent.data(), m.a_group_parent.size() * 4);
    put("group_root", m.a_group_root.data(), m.a_group_root.size() * 4);
    put("link_axis", m.a_link_axis.data(), m.a_link_axis.size() * 4);
    put("link_dof", m.a_link_dof.data(), m.a_link_dof.size() * 4);
    put("link_group", m.a_link_group.data(), m.a_link_group.size() * 4);
    put("link_inertia", m.a_link_inertia.data(), m.a_link_inertia.size() * 4);
    put("link_jtype", m.a_link_jtype.data(), m.a_link_jtype.size() * 4);
    put("link_origin", m.a_link_origin.data(), m.a_link_origin.size() * 4);
    put("link_parent", m.a_link_parent.data(), m.a_link_parent.size() * 4);
    put("shape_friction", m.a_shape_friction.data(), m.a_shape_friction.size() * 4);
    put("shape_kind", m.a_shape_kind.data(), m.a_shape_kind.size() * 4);
    put("shape_link", m.a_shape_link.data(), m.a_shape_link.size() * 4);
    put("shape_params", m.a_shape_params.data(), m.a_shape_params.size() * 4);
    put("shape_pose", m.a_shape_pose.data(), m.a_shape_pose.size() * 4);
    unsigned char dg[20];
    h.digest(dg);
    uint64_t v = 0;
    for (int i = 7; i >= 0; --i) v = v << 8 | dg[i];
    m.hash = v;
}

// ------------------------------------------------------------------ codegen (model/codegen.py emit)
std::string f9(double x) {   // codegen._f: %.9g, a '.0' when integral, 'f'
    char b[64];
    std::snprintf(b, sizeof b, "%.9g", x);
    std::string s = b;
    if (s.find('.') == std::string::npos && s.find('e') == std::string::npos && s.find("inf") == std::string::npos &&
        s.find("nan") == std::string::npos)
        s += ".0";
    return s + "f";
}
template <class T, class F> std::string arr(const std::vector<T> &v, F fmt) {
    std::string s = "{";
    for (size_t i = 0; i < v.size(); ++i) {
        if (i) s += ", ";
        s += fmt(v[i]);
    }
    return s + "}";
}
std::string iarr(const std::vector<int> &v) {
    return arr(v, [](int x) { return std::to_string(x); });
}
std::string farr(const std::vector<double> &v) {
    return arr(v, [](double x) { return f9(x); });
}
std::string sarr(const std::vector<std::string> &v) {
    return arr(v, [](const std::string &x) { return x; });
}

// joint-aligned group frame (codegen.axis_frame): Q with the unit axis as column 2
void axis_frame(const double *a0, double *Q) {
    double a[3] = {a0[0], a0[1], a0[2]};
    const double n = std::sqrt(a[0] * a[0] + a[1] * a[1] + a[2] * a[2]);
    for (double &x : a) x /= n;
    const double e[3] = {0, 0, 1};
    bool close = true;
    for (int k = 0; k < 3; ++k)
        if (!(std::fabs(a[k] - e[k]) <= 1e-8 + 1e-5 * std::fabs(e[k]))) close = false;
    if (close) {
        const double I[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
        std::memcpy(Q, I, sizeof I);
        return;
    }
    const double ref[3] = {std::fabs(a[0]) < 0.9 ? 1.0 : 0.0, std::fabs(a[0]) < 0.9 ? 0.0 : 1.0, 0.0};
    double b1[3] = {ref[1] * a[2] - ref[2] * a[1], ref[2] * a[0] - ref[0] * a[2], ref[0] * a[1] - ref[1] * a[0]};
    const double nb = std::sqrt(b1[0] * b1[0] + b1[1] * b1[1] + b1[2] * b1[2]);
    for (double &x : b1) x /= nb;
    const double b2[3] = {a[1] * b1[2] - a[2] * b1[1], a[2] * b1[0] - a[0] * b1[2], a[0] * b1[1] - a[1] * b1[0]};
    for (int r = 0; r < 3; ++r) {
        Q[3 * r] = b1[r];
        Q[3 * r + 1] = b2[r];
        Q[3 * r + 2] = a[r];
    }
}

// codegen.lane_schedule: greedy list schedule of the non-root groups onto
// `lanes` slots, longest path to a leaf first
std::vector<std::vector<int>> lane_schedule(const std::vector<int> &parent, int lanes) {
    const int G = (int)parent.size();
    std::vector<int> height(G, 0);
    for (int g = G - 1; g > 0; --g) height[parent[g]] = std::max(height[parent[g]], height[g] + 1);
    std::vector<int> step_of(G, -2);
    step_of[0] = -1;
    std::vector<std::vector<int>> steps;
    int todo = G - 1;
    while (todo > 0) {
        const int t = (int)steps.size();
        std::vector<int> ready;
        for (int g = 1; g < G; ++g)
            if (step_of[g] == -2 && step_of[parent[g]] != -2 && step_of[parent[g]] < t) ready.push_back(g);
        std::sort(ready.begin(), ready.end(), [&](int x, int y) {
            return height[x] != height[y] ? height[x] > height[y] : x < y;
        });
        std::vector<int> cur(ready.begin(), ready.begin() + std::min((int)ready.size(), lanes));
        for (int g : cur) {
            step_of[g] = t;
            --todo;
        }
        while ((int)cur.size() < lanes) cur.push_back(-1);
        steps.push_back(cur);
    }
    if (steps.empty()) steps.push_back(std::vector<int>(lanes, -1));
    return steps;
}

std::string emit(const tg_model &m) {
    const int G = (int)m.group_root.size(), L = (int)m.links.size(), D = (int)m.dof_names.size(),
              S = (int)m.shapes.size();
    std::vector<int> gdof(G), gtype(G), sgroup, nrows_n, gpar(m.group_parent.begin(), m.group_parent.end());
    std::vector<double> gaxis, gq;
    for (int g = 0; g < G; ++g) {
        const int r = m.group_root[g];
        gdof[g] = g > 0 ? m.a_link_dof[r] : -1;
        gtype[g] = g > 0 ? m.a_link_jtype[r] : 0;
        double ax[3], Q[9];
        for (int k = 0; k < 3; ++k) ax[k] = (double)m.a_link_axis[3 * r + k];
        for (int k = 0; k < 3; ++k) gaxis.push_back(ax[k]);
        if (g == 0) {
            const double I[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
            std::memcpy(Q, I, sizeof I);
        } else {
            axis_frame(ax, Q);
        }
        for (int k = 0; k < 9; ++k) gq.push_back(Q[k]);
    }
    for (int s = 0; s < S; ++s) {
        sgroup.push_back(m.a_link_group[m.a_shape_link[s]]);
        nrows_n.push_back(m.a_shape_kind[s] == S_BOX ? 4 : 1);
    }
    std::vector<std::vector<int>> anc(G, std::vector<int>(G, 0));
    std::vector<int> depth(G, 0);
    for (int k = 0; k < G; ++k) {
        int c = 0;
        for (int g = k; g >= 0; g = gpar[g]) {
            anc[k][g] = 1;
            ++c;
        }
        depth[k] = c - 1;
    }
    std::vector<int> cgroups(sgroup.begin(), sgroup.end());
    std::sort(cgroups.begin(), cgroups.end());
    cgroups.erase(std::unique(cgroups.begin(), cgroups.end()), cgroups.end());
    int maxd = 1;
    for (int c : cgroups) maxd = std::max(maxd, depth[c]);
    std::vector<std::vector<int>> cpaths;
    for (int c : cgroups) {
        std::vector<int> p;
        for (int g = 1; g < G; ++g)
            if (anc[c][g]) p.push_back(g);
        while ((int)p.size() < maxd) p.push_back(0);
        cpaths.push_back(p);
    }
    std::vector<int> shape_cg;
    for (int g : sgroup) shape_cg.push_back((int)(std::find(cgroups.begin(), cgroups.end(), g) - cgroups.begin()));
    const char *pm = std::getenv("TG_PAIR_MIN_GROUPS");
    const int SL = 8, EPB = 16, PAIR = G >= (pm ? std::atoi(pm) : 2) ? 1 : 0, LPE = SL * (1 + PAIR);
    const auto sched = lane_schedule(gpar, SL);
    std::vector<std::vector<int>> children(G);
    for (int c = 0; c < G; ++c)
        if (gpar[c] >= 0) children[gpar[c]].push_back(c);
    std::vector<int> level(L, 0), wdepth(L, 0);
    std::set<int> groot(m.group_root.begin(), m.group_root.end());
    for (int l = 0; l < L; ++l) {
        level[l] = groot.count(l) ? 0 : level[m.a_link_parent[l]] + 1;
        wdepth[l] = m.a_link_parent[l] < 0 ? 0 : wdepth[m.a_link_parent[l]] + 1;
    }
    std::vector<std::vector<int>> glinks(G);
    for (int l = 0; l < L; ++l) glinks[m.a_link_group[l]].push_back(l);
    int maxgl = 0, maxc = 1;
    for (const auto &x : glinks) maxgl = std::max(maxgl, (int)x.size());
    for (const auto &c : children) maxc = std::max(maxc, (int)c.size());
    // run-time models carry no fused task epilogue: no translating locks
    const int KX = 0, NTL = 0, lcom = (3 * L + 3) & ~3;
    auto rows = [](const std::vector<std::vector<int>> &v) {
        std::vector<std::string> r;
        for (const auto &x : v) r.push_back(iarr(x));
        return sarr(r);
    };
    auto frows = [](const std::vector<float> &v, int w, int n) {
        std::vector<std::string> r;
        for (int i = 0; i < n; ++i) r.push_back(farr(std::vector<double>(v.begin() + w * i, v.begin() + w * (i + 1))));
        return sarr(r);
    };
    auto drows = [](const std::vector<double> &v, int w, int n) {
        std::vector<std::string> r;
        for (int i = 0; i < n; ++i) r.push_back(farr(std::vector<double>(v.begin() + w * i, v.begin() + w * (i + 1))));
        return sarr(r);
    };
    std::vector<int> lp(m.a_link_parent.begin(), m.a_link_parent.end()), lg(m.a_link_group.begin(), m.a_link_group.end()),
        ld(m.a_link_dof.begin(), m.a_link_dof.end()), lj(m.a_link_jtype.begin(), m.a_link_jtype.end()),
        sl(m.a_shape_link.begin(), m.a_shape_link.end()), sk(m.a_shape_kind.begin(), m.a_shape_kind.end()),
        gp(m.a_group_parent.begin(), m.a_group_parent.end()), gr(m.a_group_root.begin(), m.a_group_root.end()),
        dl(m.a_dof_locked.begin(), m.a_dof_locked.end());
    std::vector<int> is_root(L, 0), nchild(G), cpl;
    for (int l = 0; l < L; ++l) is_root[l] = groot.count(l) ? 1 : 0;
    for (int g = 0; g < G; ++g) nchild[g] = (int)children[g].size();
    for (int c : cgroups) cpl.push_back(depth[c]);
    std::vector<std::vector<int>> childp(G), glp(G);
    for (int g = 0; g < G; ++g) {
        childp[g] = children[g];
        while ((int)childp[g].size() < maxc) childp[g].push_back(-1);
        glp[g] = glinks[g];
        while ((int)glp[g].size() < maxgl) glp[g].push_back(-1);
    }
    std::vector<float> sp = m.a_shape_params, spose = m.a_shape_pose;
    if (S == 0) {
        sp.assign(4, 0.f);
        spose.assign(12, 0.f);
    }
    char hx[32];
    std::snprintf(hx, sizeof hx, "0x%016llxULL", (unsigned long long)m.hash);
    const int NSA = std::max(S, 1);
    std::vector<int> nrows_or = nrows_n.empty() ? std::vector<int>{0} : nrows_n;
    int nrows = 0;
    for (int n : nrows_n) nrows += n + (n == 1 ? 2 : 3);   // (one-point shapes: no torsion row)
    std::vector<std::string> L_;
    auto add = [&](const std::string &x) { L_.push_back(x); };
    auto I = [](long v) { return std::to_string(v); };
    add("// AUTO-GENERATED by thormang_isaacgym_amd/model/codegen.py from model '" + m.name + "'. Do not edit.");
    add("#pragma once");
    add("struct " + m.cname + " {");
    add(std::string("  static constexpr unsigned long long hash = ") + hx + ";");
    add("  static constexpr int NG = " + I(G) + ", NL = " + I(L) + ", ND = " + I(D) + ", NS = " + I(S) + ", NSA = " + I(NSA) + ";");
    add("  static constexpr int KC = " + I(24 * G + 12 * S + KX + lcom) + ";  // per-env composite floats (env-major, csrc CompLayout)");
    add("  static constexpr int KX = " + I(KX) + ";  // of which the translating-lock extension (codegen translating_locks)");
    add("  static constexpr int LCOM = " + I(lcom ? 1 : 0) + ";  // link coms in their group frames (rigid-body force reduction)");
    add("  static constexpr int NTL = " + I(NTL) + ", tl_group = 0, NAG = 0, NASH = 0;");
    add("  static constexpr int tl_link[1] = {0};");
    add("  static constexpr int tl_dof[1] = {0};");
    add("  static constexpr int link_tl[" + I(L) + "] = " + iarr(std::vector<int>(L, 0)) + ";");
    add("  static constexpr int ag_group[1] = {0};");
    add("  static constexpr int ag_mask[1] = {0};");
    add("  static constexpr int ash_shape[1] = {0};");
    add("  static constexpr int ash_mask[1] = {0};");
    add("  static constexpr int NROWS = " + I(nrows) + ";  // contact rows (normals + 3 friction per shape, 2 for one-point shapes)");
    add("  static constexpr int parent[" + I(G) + "] = " + iarr(gp) + ";");
    add("  static constexpr int gdof[" + I(G) + "] = " + iarr(gdof) + ";");
    add("  static constexpr int jtype[" + I(G) + "] = " + iarr(gtype) + ";");
    add("  static constexpr float axis[" + I(G) + "][3] = " + drows(gaxis, 3, G) + ";");
    add("  static constexpr float gq[" + I(G) + "][9] = " + drows(gq, 9, G) + ";  // joint-aligned frames");
    add("  static constexpr int shape_group[" + I(NSA) + "] = " + iarr(sgroup.empty() ? std::vector<int>{0} : sgroup) + ";");
    add("  static constexpr int shape_kind[" + I(NSA) + "] = " + iarr(sk.empty() ? std::vector<int>{0} : sk) + ";");
    add("  static constexpr int shape_nrows[" + I(NSA) + "] = " + iarr(nrows_or) + ";");
    add("  static constexpr float shape_params[" + I(NSA) + "][4] = " + frows(sp, 4, NSA) + ";");
    add("  static constexpr float root_com[3] = " + farr({(double)m.a_link_inertia[1], (double)m.a_link_inertia[2], (double)m.a_link_inertia[3]}) + ";");
    add("  static constexpr int link_parent[" + I(L) + "] = " + iarr(lp) + ";");
    add("  static constexpr int link_group[" + I(L) + "] = " + iarr(lg) + ";");
    add("  static constexpr int link_dof[" + I(L) + "] = " + iarr(ld) + ";");
    add("  static constexpr int link_jtype[" + I(L) + "] = " + iarr(lj) + ";");
    add("  static constexpr int link_is_group_root[" + I(L) + "] = " + iarr(is_root) + ";");
    add("  static constexpr float link_origin[" + I(L) + "][12] = " + frows(m.a_link_origin, 12, L) + ";");
    add("  static constexpr float link_axis[" + I(L) + "][3] = " + frows(m.a_link_axis, 3, L) + ";");
    add("  static constexpr float link_inertia[" + I(L) + "][10] = " + frows(m.a_link_inertia, 10, L) + ";");
    add("  static constexpr int shape_link[" + I(NSA) + "] = " + iarr(sl.empty() ? std::vector<int>{0} : sl) + ";");
    add("  static constexpr float shape_pose[" + I(NSA) + "][12] = " + frows(spose, 12, NSA) + ";");
    add("  static constexpr int group_root[" + I(G) + "] = " + iarr(gr) + ";");
    add("  static constexpr unsigned char anc[" + I(G) + "][" + I(G) + "] = " + rows(anc) + ";");
    add("  static constexpr int NCG = " + I(std::max((int)cgroups.size(), 1)) + ", MAXD = " + I(maxd) + ";");
    add("  static constexpr int cgroup[" + I(std::max((int)cgroups.size(), 1)) + "] = " + iarr(cgroups.empty() ? std::vector<int>{0} : cgroups) + ";");
    add("  static constexpr int cpath_len[" + I(std::max((int)cgroups.size(), 1)) + "] = " + iarr(cpl.empty() ? std::vector<int>{0} : cpl) + ";");
    add("  static constexpr int cpath[" + I(std::max((int)cgroups.size(), 1)) + "][" + I(maxd) + "] = " +
        (cpaths.empty() ? "{" + iarr(std::vector<int>(maxd, 0)) + "}" : rows(cpaths)) + ";");
    add("  static constexpr int shape_cg[" + I(NSA) + "] = " + iarr(shape_cg.empty() ? std::vector<int>{0} : shape_cg) + ";");
    add("  static constexpr int SL = " + I(SL) + ", PAIR = " + I(PAIR) + ", LPE = " + I(LPE) + ", EPB = " + I(EPB) +
        ", NSTEP = " + I((long)sched.size()) + ", MAXC = " + I(maxc) + ";");
    add("  static constexpr int FUSED = 0;  // fused task epilogues: 1 walk, 2 Gogoro; 4 paper in-place seat");
    add("  static constexpr int sched[" + I((long)sched.size()) + "][" + I(SL) + "] = " + rows(sched) + ";");
    add("  static constexpr int nchild[" + I(G) + "] = " + iarr(nchild) + ";");
    add("  static constexpr int child[" + I(G) + "][" + I(maxc) + "] = " + rows(childp) + ";");
    add("  static constexpr int dof_locked[" + I(D) + "] = " + iarr(dl) + ";");
    int nlev = 0, ndep = 0;
    for (int l = 0; l < L; ++l) {
        nlev = std::max(nlev, level[l]);
        ndep = std::max(ndep, wdepth[l]);
    }
    add("  static constexpr int NLEV = " + I(nlev) + ", MAXGL = " + I(maxgl) + ";");
    add("  static constexpr int link_level[" + I(L) + "] = " + iarr(level) + ";");
    add("  static constexpr int NDEPTH = " + I(ndep) + ";");
    add("  static constexpr int link_depth[" + I(L) + "] = " + iarr(wdepth) + ";");
    std::vector<int> gnl;
    for (const auto &x : glinks) gnl.push_back((int)x.size());
    add("  static constexpr int group_nlinks[" + I(G) + "] = " + iarr(gnl) + ";");
    add("  static constexpr int group_links[" + I(G) + "][" + I(maxgl) + "] = " + rows(glp) + ";");
    add("};");
    add("");
    std::string out;
    for (size_t i = 0; i < L_.size(); ++i) {
        if (i) out += "\n";
        out += L_[i];
    }
    return out;
}

thread_local std::string g_model_err;

}  // namespace

extern "C" {

int tg_model_parse(const char *urdf_path, const char *name, const char *const *locked_joints, int32_t num_locked,
                   const char *mesh_root, tg_model **out) {
    if (!urdf_path || !out || num_locked < 0 || (num_locked > 0 && !locked_joints)) {
        g_model_err = "tg_model_parse: bad argument";
        return TG_ERR_ARG;
    }
    *out = nullptr;
    std::string nm = name && *name ? name : urdf_path;
    if (!(name && *name)) {   // the file's stem, as model/urdf.py load_asset names it
        nm = nm.substr(nm.find_last_of('/') + 1);
        nm = nm.substr(0, nm.find_last_of('.'));
    }
    std::vector<std::string> lk;
    for (int i = 0; i < num_locked; ++i) {
        if (!locked_joints[i]) {
            g_model_err = "tg_model_parse: null locked-joint name";
            return TG_ERR_ARG;
        }
        lk.emplace_back(locked_joints[i]);
    }
    tg_model *m = new tg_model;
    std::string err;
    if (!build_model(urdf_path, nm, lk, mesh_root ? mesh_root : "", *m, err)) {
        delete m;
        g_model_err = err;
        return TG_ERR_MODEL;
    }
    build_arrays(*m);
    char cn[40];
    std::snprintf(cn, sizeof cn, "Model_jit_%016llx", (unsigned long long)m->hash);
    m->cname = cn;
    m->source = emit(*m);
    *out = m;
    return 0;
}

int tg_model_load(const char *urdf_path, const char *name, const char *const *locked_joints, int32_t num_locked,
                  const char *mesh_root, const char *cache_dir, tg_model **out) {
    if (int rc = tg_model_parse(urdf_path, name, locked_joints, num_locked, mesh_root, out)) return rc;
    tg_model *m = *out;
    // a compiled-in specialisation needs no run-time compile
    const uint64_t n = tg_compiled_model_hashes(nullptr, 0);
    std::vector<uint64_t> hs(n ? n : 1);
    tg_compiled_model_hashes(hs.data(), (int32_t)n);
    if (std::find(hs.begin(), hs.begin() + n, m->hash) != hs.begin() + n) return 0;
    if (int rc = tg_model_jit(m->hash, m->cname.c_str(), m->source.c_str(), nullptr, cache_dir)) {
        g_model_err = tg_last_error();
        tg_model_free(m);
        *out = nullptr;
        return rc;
    }
    return 0;
}

int tg_model_get_desc(const tg_model *m, tg_model_desc *d) {
    if (!m || !d) return TG_ERR_ARG;
    std::memset(d, 0, sizeof *d);
    d->num_links = (int32_t)m->links.size();
    d->num_dofs = (int32_t)m->dof_names.size();
    d->num_groups = (int32_t)m->group_root.size();
    d->num_shapes = (int32_t)m->shapes.size();
    d->link_parent = m->a_link_parent.data();
    d->link_group = m->a_link_group.data();
    d->link_dof = m->a_link_dof.data();
    d->link_jtype = m->a_link_jtype.data();
    d->link_origin = m->a_link_origin.data();
    d->link_axis = m->a_link_axis.data();
    d->link_inertia = m->a_link_inertia.data();
    d->group_root = m->a_group_root.data();
    d->group_parent = m->a_group_parent.data();
    d->dof_locked = m->a_dof_locked.data();
    d->shape_link = m->a_shape_link.data();
    d->shape_kind = m->a_shape_kind.data();
    d->shape_pose = m->a_shape_pose.data();
    d->shape_params = m->a_shape_params.data();
    d->shape_friction = m->a_shape_friction.data();
    d->model_hash = m->hash;
    return 0;
}

const char *tg_model_dof_name(const tg_model *m, int32_t dof) {
    if (!m || dof < 0 || dof >= (int32_t)m->dof_names.size()) return nullptr;
    return m->dof_names[dof].c_str();
}

const char *tg_model_link_name(const tg_model *m, int32_t link) {
    if (!m || link < 0 || link >= (int32_t)m->links.size()) return nullptr;
    return m->links[link].name.c_str();
}

int tg_model_dof_limits(const tg_model *m, int32_t dof, float *lower, float *upper, float *effort, float *velocity) {
    if (!m || dof < 0 || dof >= (int32_t)m->dof_names.size()) return TG_ERR_ARG;
    const Joint &j = m->joints[m->dof_joint[dof]];
    if (lower) *lower = j.has_limits ? (float)j.lower : -3.4e38f;
    if (upper) *upper = j.has_limits ? (float)j.upper : 3.4e38f;
    if (effort) *effort = (float)j.effort;
    if (velocity) *velocity = (float)j.velocity;
    return 0;
}

const char *tg_model_source(const tg_model *m) { return m ? m->source.c_str() : nullptr; }

const char *tg_model_last_error(void) { return g_model_err.c_str(); }

void tg_model_free(tg_model *m) { delete m; }

}  // extern "C"
