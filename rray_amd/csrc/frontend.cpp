// frontend.cpp — drop-in front-end: scene_builder_yaml.rs (YAML -> scene registry + camera),
// load_obj.rs (+ tobj 4.0.2 semantics), canvas.rs quantisation, render_scene_from_file.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <limits>
#include <sstream>
#include <string>
#include <vector>

#include "../../include/rray/rray.h"
#include "png.hpp"
#include "rr_math.hpp"
#include "yaml.hpp"

using rr::yaml::Node;

void rr_set_error(const char* msg);  // api.cpp

struct rr_scene {
    // registry (object/db.rs) in creation order; ids index every array
    std::vector<int32_t> kind, parent, material, child_start, child_count, children, top;
    std::vector<std::vector<int32_t>> kids;
    std::vector<double> transform, tri;
    std::vector<double> mat;
    std::vector<int32_t> mat_pattern;
    std::vector<int32_t> pat_kind, pat_a, pat_b;
    std::vector<double> pat_color, pat_scale, pat_transform;
    std::vector<int32_t> pat_octaves;
    std::vector<double> pat_persistence;
    std::vector<int32_t> tex_size;  // width, height per texture
    std::vector<uint8_t> texels;    // RGBA8, textures back to back
    std::vector<std::pair<std::string, int>> tex_of_path;  // one decode per file
    std::vector<int32_t> light_kind, light_level;
    std::vector<double> light;
    std::vector<double> shape;      // minimum, maximum, closed per object (cylinder / cone)
    std::vector<int32_t> csg_op;    // per object (CSG)
    rr_scene_desc desc{};

    void finalize() {
        child_start.assign(kind.size(), 0);
        child_count.assign(kind.size(), 0);
        children.clear();
        for (size_t i = 0; i < kind.size(); ++i) {
            child_start[i] = (int32_t)children.size();
            child_count[i] = (int32_t)kids[i].size();
            children.insert(children.end(), kids[i].begin(), kids[i].end());
        }
        desc = rr_scene_desc{};
        desc.n_objects = (int32_t)kind.size();
        desc.kind = kind.data();
        desc.parent = parent.data();
        desc.transform = transform.data();
        desc.inverse = nullptr;
        desc.material = material.data();
        desc.tri = tri.data();
        desc.child_start = child_start.data();
        desc.child_count = child_count.data();
        desc.children = children.data();
        desc.n_top = (int32_t)top.size();
        desc.top = top.data();
        desc.n_materials = (int32_t)mat_pattern.size();
        desc.mat = mat.data();
        desc.mat_pattern = mat_pattern.data();
        desc.n_patterns = (int32_t)pat_kind.size();
        desc.pat_kind = pat_kind.data();
        desc.pat_a = pat_a.data();
        desc.pat_b = pat_b.data();
        desc.pat_color = pat_color.data();
        desc.pat_scale = pat_scale.data();
        desc.pat_transform = pat_transform.data();
        desc.n_lights = (int32_t)light_kind.size();
        desc.light_kind = light_kind.data();
        desc.light = light.data();
        desc.light_level = light_level.data();
        desc.shape = shape.data();
        desc.csg_op = csg_op.data();
        desc.pat_octaves = pat_octaves.data();
        desc.pat_persistence = pat_persistence.data();
        desc.n_textures = (int32_t)(tex_size.size() / 2);
        desc.tex_size = tex_size.data();
        desc.texels = texels.data();
    }
};

namespace {

struct SceneError {
    int code;
    std::string msg;
};
[[noreturn]] void panic(const std::string& m, int code = RR_E_SCENE) { throw SceneError{code, m}; }

// scene_builder_yaml.rs:68-82
double get_f64(const Node& n) {
    if (n.kind == Node::Integer) return (double)n.i;
    if (n.kind == Node::Real) {
        double d;
        if (!rr::yaml::rust_parse_f64(n.s, d)) panic("'" + n.s + "' is not a valid f64");
        return d;
    }
    panic("not a number");
}
double get_f64_default(const Node& n, double def) {
    if (n.kind == Node::Integer || n.kind == Node::Real) return get_f64(n);
    return def;
}
const std::vector<Node>& as_vec(const Node& n, const char* what) {
    if (n.kind != Node::Array) panic(std::string(what) + " not found");
    return n.seq;
}
rr::Tup tuple3(const Node& n, double w, const char* what) {
    const auto& v = as_vec(n, what);
    if (v.size() < 3) panic(std::string(what) + ": expected 3 numbers");
    return {get_f64(v[0]), get_f64(v[1]), get_f64(v[2]), w};
}
double deg2rad(double d) { return d * M_PI / 180.0; }  // :25-27

rr::M4 create_matrix(const Node& t) {  // :178-216
    const Node& ty = t["type"];
    if (ty.kind != Node::String) panic("transform type not found");
    if (ty.s == "translate" || ty.s == "scale") {
        const auto& a = as_vec(t["amount"], "amount");
        if (a.size() < 3) panic("amount: expected 3 numbers");
        double x = get_f64(a[0]), y = get_f64(a[1]), z = get_f64(a[2]);
        return ty.s == "translate" ? rr::translate(x, y, z) : rr::scale(x, y, z);
    }
    if (ty.s == "rotate") {
        double ang = deg2rad(get_f64(t["angle"]));
        const Node& axis = t["axis"];
        if (axis.kind != Node::String) panic("axis not found");
        if (axis.s == "x") return rr::rotate(0, ang);
        if (axis.s == "y") return rr::rotate(1, ang);
        if (axis.s == "z") return rr::rotate(2, ang);
        panic("Unknown axis: " + axis.s);
    }
    if (ty.s == "shear")
        return rr::shear(get_f64(t["xy"]), get_f64(t["xz"]), get_f64(t["yx"]), get_f64(t["yz"]), get_f64(t["zx"]),
                         get_f64(t["zy"]));
    panic("Unknown transform type: " + ty.s);
}
rr::M4 create_transforms(const Node& ts) {  // :218-224 (reversed, m = m * T)
    rr::M4 m = rr::identity();
    if (ts.kind != Node::Array) return m;
    for (size_t k = ts.seq.size(); k-- > 0;) m = rr::multiply(m, create_matrix(ts.seq[k]));
    return m;
}

struct Builder {
    rr_scene& S;
    std::string obj_root;

    int add_pattern(int kind, const rr::M4& m, double r = 0, double g = 0, double b = 0, int a = -1, int bb = -1,
                    double scale = 0.5, int32_t octaves = 1, double persistence = 1.0) {
        S.pat_kind.push_back(kind);
        S.pat_a.push_back(a);
        S.pat_b.push_back(bb);
        S.pat_color.insert(S.pat_color.end(), {r, g, b});
        S.pat_scale.push_back(scale);
        S.pat_transform.insert(S.pat_transform.end(), m.m, m.m + 16);
        S.pat_octaves.push_back(octaves);
        S.pat_persistence.push_back(persistence);
        return (int)S.pat_kind.size() - 1;
    }
    int create_pattern(const Node& p) {  // :226-308
        rr::M4 transform = create_transforms(p["transforms"]);
        const Node& ty = p["type"];
        if (ty.kind != Node::String) panic("pattern type not found");
        const Node& color = p["color"];
        rr::Tup c = color.is_bad() ? rr::Tup{0, 0, 0, 0} : tuple3(color, 0, "color");
        if (ty.s == "solid") return add_pattern(RR_PAT_SOLID, transform, c.x, c.y, c.z);
        int kind = ty.s == "stripe"     ? RR_PAT_STRIPE
                   : ty.s == "gradient" ? RR_PAT_GRADIENT
                   : ty.s == "ring"     ? RR_PAT_RING
                   : ty.s == "checker"  ? RR_PAT_CHECKER
                   : ty.s == "blend"    ? RR_PAT_BLEND
                                        : -1;
        if (kind >= 0) {
            double scale = kind == RR_PAT_BLEND ? get_f64_default(p["scale"], 0.5) : 0.5;
            int a = sub_pattern(transform, p["color_a"], p["pattern_a"]);
            int b = sub_pattern(transform, p["color_b"], p["pattern_b"]);
            return add_pattern(kind, transform, 0, 0, 0, a, b, scale);
        }
        if (ty.s == "perturbed") {  // :272-281
            double scale = get_f64_default(p["scale"], 0.2);
            int32_t octaves = as_octaves(get_f64_default(p["octaves"], 3.0));
            double persistence = get_f64_default(p["persistence"], 0.5);
            int a = sub_pattern(transform, p["color_a"], p["pattern_a"]);
            return add_pattern(RR_PAT_PERTURBED, transform, 0, 0, 0, a, -1, scale, octaves, persistence);
        }
        if (ty.s == "noise") {  // :282-292
            int32_t octaves = as_octaves(get_f64_default(p["octaves"], 1.0));
            double persistence = get_f64_default(p["persistence"], 1.0);
            double scale = get_f64_default(p["scale"], 1.0);
            int a = sub_pattern(transform, p["color_a"], p["pattern_a"]);
            int b = sub_pattern(transform, p["color_b"], p["pattern_b"]);
            return add_pattern(RR_PAT_NOISE, transform, 0, 0, 0, a, b, scale, octaves, persistence);
        }
        if (ty.s == "image") {  // :293-296 -> Texture::new (texture.rs:15-19)
            const Node& file = p["file"];
            if (file.kind != Node::String) panic("file not found");
            return add_pattern(RR_PAT_TEXTURE, transform, 0, 0, 0, load_texture(file.s));
        }
        return add_pattern(RR_PAT_SOLID, transform, 0, 0, 0);
    }
    // `f64 as usize` (saturating, NaN -> 0); counts above RR_MAX_OCTAVES are rejected at upload
    static int32_t as_octaves(double v) {
        if (!(v > 0)) return 0;
        return v >= 2147483647.0 ? 2147483647 : (int32_t)v;
    }
    int load_texture(const std::string& file) {
        std::string path = file;
        if (!obj_root.empty() && !file.empty() && file[0] != '/') path = obj_root + "/" + file;
        for (auto& e : S.tex_of_path)
            if (e.first == path) return e.second;
        std::vector<uint8_t> rgba;
        uint32_t w = 0, h = 0;
        std::string err;
        int rc = rr::read_image_rgba(path, rgba, w, h, err);
        if (rc != RR_OK) panic(err, rc);
        if (w > 0x7fffffffu || h > 0x7fffffffu) panic(path + ": texture too large", RR_E_LIMIT);
        int id = (int)(S.tex_size.size() / 2);
        S.tex_size.push_back((int32_t)w);
        S.tex_size.push_back((int32_t)h);
        S.texels.insert(S.texels.end(), rgba.begin(), rgba.end());
        S.tex_of_path.emplace_back(path, id);
        return id;
    }
    int sub_pattern(const rr::M4& t, const Node& color, const Node& pat) {  // :310-317
        if (color.is_array()) {
            rr::Tup c = tuple3(color, 0, "color");
            return add_pattern(RR_PAT_SOLID, t, c.x, c.y, c.z);
        }
        return create_pattern(pat);
    }
    int create_material(const Node& m) {  // :319-332
        double v[7] = {0.1, 0.9, 0.9, 200.0, 0.0, 0.0, 1.0};
        int pat = -1;
        if (!m.is_bad()) {
            v[0] = get_f64_default(m["ambient"], 0.1);
            v[1] = get_f64_default(m["diffuse"], 0.9);
            v[2] = get_f64_default(m["specular"], 0.9);
            v[3] = get_f64_default(m["shininess"], 200.0);
            v[4] = get_f64_default(m["reflective"], 0.0);
            v[5] = get_f64_default(m["transparency"], 0.0);
            v[6] = get_f64_default(m["refractive_index"], 1.0);
            pat = create_pattern(m["pattern"]);
        }
        S.mat.insert(S.mat.end(), v, v + 7);
        S.mat_pattern.push_back(pat);
        return (int)S.mat_pattern.size() - 1;
    }
    int new_object(int kind, int parent) {  // db.rs get_next_id + Group::add_child / Scene::add_object
        int id = (int)S.kind.size();
        S.kind.push_back(kind);
        S.parent.push_back(parent);
        S.material.push_back(-1);
        rr::M4 I = rr::identity();
        S.transform.insert(S.transform.end(), I.m, I.m + 16);
        S.tri.insert(S.tri.end(), 18, 0.0);
        S.shape.insert(S.shape.end(), {-std::numeric_limits<double>::infinity(), std::numeric_limits<double>::infinity(), 0.0});
        S.csg_op.push_back(RR_CSG_UNION);
        S.kids.emplace_back();
        if (parent >= 0)
            S.kids[parent].push_back(id);
        else
            S.top.push_back(id);
        return id;
    }
    void set_transform(int id, const rr::M4& m) { std::memcpy(&S.transform[16 * (size_t)id], m.m, sizeof(m.m)); }

    int load_obj(const std::string& path, int parent, int material);
    int create_shape(const Node& s, int parent) {  // :334-365
        const Node& ty = s["type"];
        if (ty.kind != Node::String) panic("type not found");
        const std::string& t = ty.s;
        int id;
        if (t == "sphere" || t == "glass_sphere") {
            id = new_object(RR_SPHERE, parent);
        } else if (t == "plane") {
            id = new_object(RR_PLANE, parent);
        } else if (t == "triangle") {
            rr::Tup p1 = tuple3(s["p1"], 1, "p1"), p2 = tuple3(s["p2"], 1, "p2"), p3 = tuple3(s["p3"], 1, "p3");
            id = new_object(RR_TRIANGLE, parent);
            double* d = &S.tri[18 * (size_t)id];
            const double v[9] = {p1.x, p1.y, p1.z, p2.x, p2.y, p2.z, p3.x, p3.y, p3.z};
            std::memcpy(d, v, sizeof(v));
        } else if (t == "obj_file") {
            const Node& f = s["obj_file"];
            if (f.kind != Node::String) panic("obj_file not found");
            int m = create_material(s["material"]);
            id = load_obj(f.s, parent, m);
        } else if (t == "group") {
            id = new_object(RR_GROUP, parent);
            for (const Node& ch : as_vec(s["children"], "children")) {
                const Node& h = ch["hidden"];
                if (!(h.kind == Node::Bool && h.b)) create_shape(ch, id);
            }
        } else if (t == "cube") {
            id = new_object(RR_CUBE, parent);
        } else if (t == "cylinder" || t == "cone") {  // :332-343
            const double inf = std::numeric_limits<double>::infinity();
            const double mn = get_f64_default(s["minimum"], -inf), mx = get_f64_default(s["maximum"], inf);
            const Node& cl = s["closed"];
            const bool closed = cl.kind == Node::Bool && cl.b;  // as_bool().unwrap_or(false)
            id = new_object(t == "cylinder" ? RR_CYLINDER : RR_CONE, parent);
            S.shape[3 * (size_t)id] = mn;
            S.shape[3 * (size_t)id + 1] = mx;
            S.shape[3 * (size_t)id + 2] = closed ? 1.0 : 0.0;
        } else if (t == "csg") {  // :152-162: operation, then left and right (created in that order)
            const Node& op = s["operation"];
            if (op.kind != Node::String) panic("operation not found");
            int code;
            if (op.s == "union")
                code = RR_CSG_UNION;
            else if (op.s == "intersection")
                code = RR_CSG_INTERSECTION;
            else if (op.s == "difference")
                code = RR_CSG_DIFFERENCE;
            else
                panic("Unknown operation: " + op.s);
            id = new_object(RR_CSG, parent);
            S.csg_op[id] = code;
            create_shape(s["left"], id);
            create_shape(s["right"], id);
        } else if (t == "torus") {  // :350-353
            const double r = get_f64(s["minor_radius"]);
            id = new_object(RR_TORUS, parent);
            S.shape[3 * (size_t)id] = r;
        } else {
            panic("Unknown object type: " + t);
        }
        set_transform(id, create_transforms(s["transforms"]));
        int m = create_material(s["material"]);  // Group / Csg::set_material are no-ops (group.rs, csg.rs)
        if (S.kind[id] != RR_GROUP && S.kind[id] != RR_CSG) S.material[id] = m;
        return id;
    }
};

// load_obj.rs:124-139 with tobj 4.0.2 (LoadOptions::default()) semantics: f32 positions/normals
// widened with `as f64`; `o`/`g` start a new model when faces are pending; face_arities is empty
// for an all-triangle model, so get_faces() yields nothing for it (load_obj.rs:26-40).
int Builder::load_obj(const std::string& file, int parent, int material) {
    std::string path = file;
    if (!obj_root.empty() && !file.empty() && file[0] != '/') path = obj_root + "/" + file;
    std::ifstream f(path, std::ios::binary);
    if (!f) panic("Failed to OBJ load file: " + file, RR_E_IO);
    std::stringstream ss;
    ss << f.rdbuf();
    std::string text = ss.str();
    for (auto& ch : text)
        if (ch == '\r') ch = '\n';
    struct Model {
        std::vector<std::vector<long>> fv, fn;
        bool normals = false;
    };
    std::vector<float> pos, nrm;
    std::vector<Model> models;
    Model cur;
    auto idx = [](const std::string& s, size_t n) {
        long i = std::strtol(s.c_str(), nullptr, 10);
        return i < 0 ? (long)n + i : i - 1;
    };
    std::istringstream in(text);
    std::string line;
    while (std::getline(in, line)) {
        std::istringstream ls(line);
        std::string tag;
        if (!(ls >> tag)) continue;
        if (tag == "v" || tag == "vn") {
            std::string a, b, c;
            ls >> a >> b >> c;
            auto& dst = tag == "v" ? pos : nrm;
            dst.push_back(std::strtof(a.c_str(), nullptr));  // tobj: f32
            dst.push_back(std::strtof(b.c_str(), nullptr));
            dst.push_back(std::strtof(c.c_str(), nullptr));
        } else if (tag == "f") {
            std::vector<long> fv, fn;
            std::string tok;
            while (ls >> tok) {
                size_t s1 = tok.find('/');
                fv.push_back(idx(tok.substr(0, s1), pos.size() / 3));
                if (s1 != std::string::npos) {
                    size_t s2 = tok.find('/', s1 + 1);
                    if (s2 != std::string::npos && s2 + 1 < tok.size())
                        fn.push_back(idx(tok.substr(s2 + 1), nrm.size() / 3));
                }
            }
            if (fv.size() < 3) continue;
            for (long i : fv)
                if (i < 0 || (size_t)i >= pos.size() / 3) panic("OBJ face index out of range: " + file, RR_E_IO);
            for (long i : fn)
                if (i < 0 || (size_t)i >= nrm.size() / 3) panic("OBJ normal index out of range: " + file, RR_E_IO);
            if (!fn.empty()) {
                if (fn.size() != fv.size()) panic("OBJ face with partial normals: " + file, RR_E_IO);
                cur.normals = true;
            }
            cur.fv.push_back(fv);
            cur.fn.push_back(fn);
        } else if (tag == "o" || tag == "g") {
            if (!cur.fv.empty()) models.push_back(cur);
            cur = Model();
        }
    }
    if (!cur.fv.empty()) models.push_back(cur);
    if (models.empty()) panic("No models found in file: " + file);
    auto make_group = [&](const Model& m, int par) {
        int g = new_object(RR_GROUP, par);
        bool all_tri = true;
        for (auto& fv : m.fv)
            if (fv.size() != 3) all_tri = false;
        if (all_tri) return g;
        for (size_t fi = 0; fi < m.fv.size(); ++fi) {
            const auto& fv = m.fv[fi];
            for (size_t i = 1; i + 1 < fv.size(); ++i) {  // fan (v0, vi, vi+1)
                int id = new_object(m.normals ? RR_SMOOTH_TRIANGLE : RR_TRIANGLE, g);
                S.material[id] = material;  // material.clone() per triangle
                double* d = &S.tri[18 * (size_t)id];
                const long vi[3] = {fv[0], fv[i], fv[i + 1]};
                for (int k = 0; k < 3; ++k)
                    for (int c = 0; c < 3; ++c) d[3 * k + c] = (double)pos[3 * vi[k] + c];
                if (m.normals) {
                    const auto& fn = m.fn[fi];
                    const long ni[3] = {fn[0], fn[i], fn[i + 1]};
                    for (int k = 0; k < 3; ++k)
                        for (int c = 0; c < 3; ++c) d[9 + 3 * k + c] = (double)nrm[3 * ni[k] + c];
                }
            }
        }
        return g;
    };
    if (models.size() == 1) return make_group(models[0], parent);
    int master = new_object(RR_GROUP, parent);
    for (auto& m : models) make_group(m, master);
    return master;
}

int build_scene(const std::string& text, const char* obj_root, int64_t width, int64_t height, int32_t aa,
                rr_scene* S, rr_camera* cam) {
    Node doc;
    std::string err;
    if (!rr::yaml::load_first(text, doc, err)) panic("YAML: " + err);
    // create_camera (:89-110)
    const Node& c = doc["camera"];
    if (c.kind != Node::Hash) panic("camera definition not found");
    double fov = get_f64(c["fov"]);
    rr::Tup from = tuple3(c["from"], 1, "camera.from"), to = tuple3(c["to"], 1, "camera.to"),
            up = tuple3(c["up"], 0, "camera.up");
    rr::M4 view = rr::view_transform(from, to, up);
    if (width * aa <= 0 || height * aa <= 0) panic("image size must be positive", RR_E_ARG);
    rr_camera_new(width * aa, height * aa, deg2rad(fov), view.m, cam);
    // create_lights (:112-151)
    const Node& lights = doc["lights"];
    if (lights.kind != Node::Array) panic("lights not found");
    if (lights.seq.empty()) panic("No lights found in scene");
    for (const Node& l : lights.seq) {
        const Node& ty = l["type"];
        if (ty.kind != Node::String) panic("light.light_type not found");
        rr::Tup col = tuple3(l["color"], 0, "light.color");
        double rec[15] = {0};
        rec[3] = col.x;
        rec[4] = col.y;
        rec[5] = col.z;
        if (ty.s == "point") {
            rr::Tup p = tuple3(l["position"], 1, "light.position");
            rec[0] = p.x;
            rec[1] = p.y;
            rec[2] = p.z;
            S->light_kind.push_back(RR_LIGHT_POINT);
            S->light_level.push_back(0);
        } else if (ty.s == "area") {
            rr::Tup corner = tuple3(l["corner"], 1, "corner"), u = tuple3(l["uvec"], 0, "uvec"),
                    v = tuple3(l["vvec"], 0, "vvec");
            const Node& lv = l["level"];
            int64_t level = lv.kind == Node::Integer ? lv.i : 5;  // as_i64().unwrap_or(5)
            if (level <= 0 || level > RR_MAX_AREA_LEVEL) panic("area light level out of range (1..RR_MAX_AREA_LEVEL)", RR_E_LIMIT);
            rr::Tup center = (corner + u * 0.5) + v * 0.5;  // light.rs:41-45
            const double vals[12] = {center.x, center.y, center.z, 0, 0, 0, corner.x, corner.y, corner.z, u.x, u.y, u.z};
            for (int k = 0; k < 3; ++k) rec[k] = vals[k];
            for (int k = 0; k < 6; ++k) rec[6 + k] = vals[6 + k];
            rec[12] = v.x;
            rec[13] = v.y;
            rec[14] = v.z;
            S->light_kind.push_back(RR_LIGHT_AREA);
            S->light_level.push_back((int32_t)level);
        } else {
            panic("Unknown light type: " + ty.s);
        }
        S->light.insert(S->light.end(), rec, rec + 15);
    }
    Builder B{*S, obj_root ? std::string(obj_root) : std::string()};
    const Node& scene = doc["scene"];
    if (scene.kind != Node::Array) panic("scene not found");
    for (const Node& o : scene.seq) {  // :400-406
        const Node& h = o["hidden"];
        if (!(h.kind == Node::Bool && h.b)) B.create_shape(o, -1);
    }
    S->finalize();
    return RR_OK;
}

}  // namespace

extern "C" {

int rr_scene_from_yaml(const char* yaml_text, const char* obj_root, int64_t width, int64_t height, int32_t aa,
                       rr_scene** out_scene, rr_camera* out_camera) {
    if (!yaml_text || !out_scene || !out_camera) return RR_E_ARG;
    *out_scene = nullptr;
    if (aa < 1) {
        rr_set_error("aa must be >= 1");
        return RR_E_ARG;
    }
    rr_scene* S = new rr_scene();
    try {
        build_scene(yaml_text, obj_root, width, height, aa, S, out_camera);
    } catch (const SceneError& e) {
        delete S;
        rr_set_error(e.msg.c_str());
        return e.code;
    } catch (const std::exception& e) {
        delete S;
        rr_set_error(e.what());
        return RR_E_SCENE;
    }
    *out_scene = S;
    return RR_OK;
}

const rr_scene_desc* rr_scene_desc_of(const rr_scene* s) { return s ? &s->desc : nullptr; }
void rr_scene_free(rr_scene* s) { delete s; }

int rr_quantize(const double* avg, int64_t n, uint8_t* rgba) {  // canvas.rs:97-100 (`as u8` saturates)
    if (n < 0 || (n > 0 && (!avg || !rgba))) return RR_E_ARG;
    auto q = [](double v) -> uint8_t {
        double x = v * 255.0;
        if (!(x > 0.0)) return 0;  // NaN and <= 0
        if (x >= 255.0) return 255;
        return (uint8_t)x;
    };
    for (int64_t i = 0; i < n; ++i) {
        rgba[4 * i] = q(avg[3 * i]);
        rgba[4 * i + 1] = q(avg[3 * i + 1]);
        rgba[4 * i + 2] = q(avg[3 * i + 2]);
        rgba[4 * i + 3] = 255;
    }
    return RR_OK;
}

int rr_write_png(const char* path, const uint8_t* rgba, int64_t w, int64_t h) {
    if (!path || !rgba || w <= 0 || h <= 0) return RR_E_ARG;
    return rr::write_png_rgba(path, rgba, (uint32_t)w, (uint32_t)h) ? RR_OK : RR_E_IO;
}

int rr_render_scene_from_file(const char* path, int64_t width, int64_t height, const char* png_file, int32_t aa,
                              int device) {
    return rr_render_scene_from_file_devices(path, width, height, png_file, aa, 1, &device);
}

int rr_render_scene_from_file_devices(const char* path, int64_t width, int64_t height, const char* png_file,
                                      int32_t aa, int n_devices, const int* device_ids) {
    if (n_devices < 1 || !device_ids) {
        rr_set_error("need at least one device");
        return RR_E_ARG;
    }
    std::ifstream f(path ? path : "", std::ios::binary);
    if (!path || !f) {  // scene_builder_yaml.rs:434 panics "File does not exist"
        rr_set_error("File does not exist");
        return RR_E_IO;
    }
    std::stringstream ss;
    ss << f.rdbuf();
    rr_scene* S = nullptr;
    rr_camera cam;
    int rc = rr_scene_from_yaml(ss.str().c_str(), nullptr, width, height, aa, &S, &cam);
    if (rc != RR_OK) return rc;
    rr_ctx* ctx = nullptr;
    rc = n_devices == 1 ? rr_create(device_ids[0], &ctx) : rr_create_multi(n_devices, device_ids, &ctx);
    if (rc == RR_OK) rc = rr_scene_upload(ctx, rr_scene_desc_of(S));
    std::vector<double> avg((size_t)width * height * 3);
    if (rc == RR_OK) {
        rr_render_opts o{};
        o.aa = aa;
        o.max_depth = 5;  // camera.rs:113
        o.seed = 0;
        o.jitter_mode = 0;
        o.part = 0;
        o.nparts = 1;
        o.block_rows = 8;
        o.flags = RR_OUT_AVG;
        rc = rr_render(ctx, &cam, &o, nullptr, avg.data(), nullptr);
    }
    if (rc == RR_OK) {
        std::vector<uint8_t> rgba((size_t)width * height * 4);
        rr_quantize(avg.data(), width * height, rgba.data());
        rc = rr_write_png(png_file, rgba.data(), width, height);
        if (rc != RR_OK) rr_set_error("cannot write PNG");
    }
    rr_destroy(ctx);
    rr_scene_free(S);
    return rc;
}

}  // extern "C"
