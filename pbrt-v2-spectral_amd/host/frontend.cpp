// frontend.cpp -- pbrt-v2 scene-file front end for the MI355X path tracer.
//
// Reads the unchanged pbrt scene format and builds the flattened device scene with the
// reference's semantics:
//   * tokenizer / directive grammar        core/pbrtlex.ll, core/pbrtparse.yy (numbers via
//                                          (float)atof, integers via int(float))
//   * parameter lists / typed lookups      core/paramset.cpp (color -> FromRGB reflectance)
//   * graphics state, transform stack,     core/api.cpp:146-330, 733-1330
//     transform cache, shapes, area lights
//   * shapes                               shapes/trianglemesh.cpp, shapes/loopsubdiv.cpp,
//                                          shapes/sphere.cpp, shapes/disk.cpp
//   * primitive refinement order           core/primitive.cpp:40-53 (LIFO todo list)
//   * BVH build (SAH, 12 buckets, 4 prims) accelerators/bvh.cpp:145-372
//   * camera / film extent                 cameras/perspective.cpp, core/camera.cpp:84-103,
//                                          film/spectralImage.cpp:40-50,176-185
// Float expressions keep the reference's operand order (compile with -ffp-contract=off).
#include "scene.h"
#include "pbrthost.h"
#include "eye_ior_tables.inc"
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <cctype>
#include <fstream>
#include <sstream>
#include <set>
#include <memory>
#include <stdexcept>
#include <algorithm>
#include <chrono>
#include <functional>

namespace pbrtamd {

// ------------------------------------------------------------------------------------
// Parameter sets
// ------------------------------------------------------------------------------------
enum PCat { P_INT, P_BOOL, P_FLOAT, P_POINT, P_VECTOR, P_NORMAL, P_SPECTRUM, P_STRING, P_TEXTURE, P_NCAT };
struct Param {
    PCat cat;
    std::string name;
    std::vector<float> f;             // float/point/vector/normal
    std::vector<int> i;               // int
    std::vector<bool> b;
    std::vector<std::string> s;       // string / texture
    std::vector<Spec> spec;
};
struct ParamSet {
    std::vector<Param> items;
    void Add(const Param &p) {
        for (size_t k = 0; k < items.size(); ++k)
            if (items[k].cat == p.cat && items[k].name == p.name) { items.erase(items.begin() + k); break; }
        items.push_back(p);
    }
    const Param *Find(PCat c, const std::string &n) const {
        for (const Param &p : items) if (p.cat == c && p.name == n) return &p;
        return nullptr;
    }
    float FindOneFloat(const std::string &n, float d) const { const Param *p = Find(P_FLOAT, n); return (p && p->f.size()) ? p->f[0] : d; }
    int FindOneInt(const std::string &n, int d) const { const Param *p = Find(P_INT, n); return (p && p->i.size()) ? p->i[0] : d; }
    bool FindOneBool(const std::string &n, bool d) const { const Param *p = Find(P_BOOL, n); return (p && p->b.size()) ? p->b[0] : d; }
    std::string FindOneString(const std::string &n, const std::string &d) const { const Param *p = Find(P_STRING, n); return (p && p->s.size()) ? p->s[0] : d; }
    std::string FindTexture(const std::string &n) const { const Param *p = Find(P_TEXTURE, n); return (p && p->s.size()) ? p->s[0] : ""; }
    Spec FindOneSpectrum(const std::string &n, const Spec &d) const { const Param *p = Find(P_SPECTRUM, n); return (p && p->spec.size()) ? p->spec[0] : d; }
    V3 FindOnePoint(const std::string &n, const V3 &d) const { const Param *p = Find(P_POINT, n); return (p && p->f.size() >= 3) ? V3(p->f[0], p->f[1], p->f[2]) : d; }
    V3 FindOneVector(const std::string &n, const V3 &d) const { const Param *p = Find(P_VECTOR, n); return (p && p->f.size() >= 3) ? V3(p->f[0], p->f[1], p->f[2]) : d; }
};

// texture values known at scene-build time (constant textures; 1x1 fallback images)
// non-constant ones refer to a pbrtgpu_texture (index `tex` into HostScene::textures)
struct FloatTex { bool constant = true; float value = 0.f; int tex = -1; };
struct SpecTex { bool constant = true; Spec value; int tex = -1; };

// ------------------------------------------------------------------------------------
// Tokenizer (pbrtlex.ll)
// ------------------------------------------------------------------------------------
struct Token {
    enum Kind { END, IDENT, STRING, NUMBER, LBRACK, RBRACK } kind = END;
    std::string text;
    float num = 0.f;
};
class Lexer {
public:
    bool Open(const std::string &path) {
        std::ifstream in(path);
        if (!in) return false;
        std::stringstream ss; ss << in.rdbuf();
        stack.push_back({ss.str(), 0, path});
        return true;
    }
    bool Next(Token *t) {
        while (!stack.empty()) {
            Src &s = stack.back();
            const std::string &b = s.buf;
            size_t &p = s.pos;
            while (p < b.size()) {
                char c = b[p];
                if (isspace((unsigned char)c)) { ++p; continue; }
                if (c == '#') { while (p < b.size() && b[p] != '\n') ++p; continue; }
                if (c == '[') { ++p; t->kind = Token::LBRACK; return true; }
                if (c == ']') { ++p; t->kind = Token::RBRACK; return true; }
                if (c == '"') {
                    ++p;
                    std::string str;
                    while (p < b.size() && b[p] != '"') {
                        if (b[p] == '\\' && p + 1 < b.size()) {
                            ++p;
                            char e = b[p];
                            switch (e) {
                                case 'n': str += '\n'; break; case 't': str += '\t'; break;
                                case 'b': str += '\b'; break; case 'f': str += '\f'; break;
                                case 'r': str += '\r'; break; case '\n': break;
                                default: str += e;
                            }
                            ++p;
                            continue;
                        }
                        str += b[p++];
                    }
                    ++p;
                    t->kind = Token::STRING; t->text = str; return true;
                }
                if (isdigit((unsigned char)c) || c == '-' || c == '+' || c == '.') {
                    size_t q = p;
                    if (b[q] == '-' || b[q] == '+') ++q;
                    while (q < b.size() && (isdigit((unsigned char)b[q]) || b[q] == '.')) ++q;
                    if (q < b.size() && (b[q] == 'e' || b[q] == 'E')) {
                        size_t r = q + 1;
                        if (r < b.size() && (b[r] == '-' || b[r] == '+')) ++r;
                        if (r < b.size() && isdigit((unsigned char)b[r])) { q = r; while (q < b.size() && isdigit((unsigned char)b[q])) ++q; }
                    }
                    t->kind = Token::NUMBER; t->text = b.substr(p, q - p);
                    t->num = (float)atof(t->text.c_str());   // pbrtlex.ll:150
                    p = q;
                    return true;
                }
                if (isalpha((unsigned char)c) || c == '_') {
                    size_t q = p;
                    while (q < b.size() && (isalnum((unsigned char)b[q]) || b[q] == '_')) ++q;
                    t->kind = Token::IDENT; t->text = b.substr(p, q - p);
                    p = q;
                    return true;
                }
                throw std::runtime_error(std::string("illegal character in ") + s.path);
            }
            stack.pop_back();   // end of an included file
        }
        t->kind = Token::END;
        return false;
    }
    bool Include(const std::string &path) { return Open(path); }
private:
    struct Src { std::string buf; size_t pos; std::string path; };
    std::vector<Src> stack;
};

// ------------------------------------------------------------------------------------
// Scene builder state (api.cpp)
// ------------------------------------------------------------------------------------
struct ShapeObj;   // a (possibly refinable) shape
struct TriMesh {
    Xform o2w;            // ObjectToWorld (cached transform value)
    bool ro = false, swaps = false;
    int ntris = 0, nverts = 0;
    std::vector<int> vi;
    std::vector<V3> p;    // world space (trianglemesh.cpp:61-62)
    std::vector<V3> n;    // object space normals
    std::vector<float> uv;
    int flatIndex = -1;   // index into HostScene::meshes once emitted
};
struct Quadric {
    pbrtgpu_quadric q{};
    Xform o2w;
    BBox ObjectBound() const {
        if (q.type == PBRTGPU_SHAPE_SPHERE || q.type == PBRTGPU_SHAPE_CYLINDER)   // cylinder.cpp:40-44
            return BBox(V3(-q.radius, -q.radius, q.zmin), V3(q.radius, q.radius, q.zmax));
        return BBox(V3(-q.radius, -q.radius, q.height), V3(q.radius, q.radius, q.height));
    }
    float Area() const {
        if (q.type == PBRTGPU_SHAPE_SPHERE) return q.phi_max * q.radius * (q.zmax - q.zmin);
        if (q.type == PBRTGPU_SHAPE_CYLINDER) return (q.zmax - q.zmin) * q.phi_max * q.radius;   // cylinder.cpp:180-182
        return q.phi_max * 0.5f * (q.radius * q.radius - q.inner_radius * q.inner_radius);
    }
    int flatIndex = -1;
};
struct LoopSubdivShape;
// NURBS evaluation (nurbs.cpp:33-141), in the reference's float operations and order: the
// de Boor triangle over one knot span of homogeneous control points, the derivative from the last
// step.  Control point k of a call is cp[k * stride - bias] (the reference offsets the pointer).
struct NurbsH3 { float x = 0.f, y = 0.f, z = 0.f, w = 0.f; };
static int NurbsKnotOffset(const float *knot, int order, float t) {
    int k = order - 1;
    while (t > knot[k + 1]) ++k;
    return k;
}
static NurbsH3 NurbsEvaluate(int order, const float *knot, const NurbsH3 *cp, int bias, int cpStride, float t, V3 *deriv) {
    const int ko = NurbsKnotOffset(knot, order, t);
    knot += ko;
    const int cpOffset = ko - order + 1;
    std::vector<NurbsH3> w(order);
    for (int i = 0; i < order; ++i) w[i] = cp[(cpOffset + i) * cpStride - bias];
    for (int i = 0; i < order - 2; ++i)
        for (int j = 0; j < order - 1 - i; ++j) {
            const float alpha = (knot[1 + j] - t) / (knot[1 + j] - knot[j + 2 - order + i]);
            w[j].x = w[j].x * alpha + w[j + 1].x * (1 - alpha);
            w[j].y = w[j].y * alpha + w[j + 1].y * (1 - alpha);
            w[j].z = w[j].z * alpha + w[j + 1].z * (1 - alpha);
            w[j].w = w[j].w * alpha + w[j + 1].w * (1 - alpha);
        }
    const float alpha = (knot[1] - t) / (knot[1] - knot[0]);
    NurbsH3 val;
    val.x = w[0].x * alpha + w[1].x * (1 - alpha);
    val.y = w[0].y * alpha + w[1].y * (1 - alpha);
    val.z = w[0].z * alpha + w[1].z * (1 - alpha);
    val.w = w[0].w * alpha + w[1].w * (1 - alpha);
    if (deriv) {
        const float factor = (order - 1) / (knot[1] - knot[0]);
        const float dx = (w[1].x - w[0].x) * factor, dy = (w[1].y - w[0].y) * factor, dz = (w[1].z - w[0].z) * factor,
                    dw = (w[1].w - w[0].w) * factor;
        deriv->x = dx / val.w - (val.x * dw / (val.w * val.w));
        deriv->y = dy / val.w - (val.y * dw / (val.w * val.w));
        deriv->z = dz / val.w - (val.z * dw / (val.w * val.w));
    }
    return val;
}
static V3 NurbsEvaluateSurface(int uOrder, const float *uKnot, int ucp, float u, int vOrder, const float *vKnot, int vcp,
                               float v, const NurbsH3 *cp, V3 *dPdu, V3 *dPdv) {
    std::vector<NurbsH3> iso(std::max(uOrder, vOrder));
    const int uFirstCp = NurbsKnotOffset(uKnot, uOrder, u) - uOrder + 1;
    for (int i = 0; i < uOrder; ++i) iso[i] = NurbsEvaluate(vOrder, vKnot, cp + uFirstCp + i, 0, ucp, v, nullptr);
    const int vFirstCp = NurbsKnotOffset(vKnot, vOrder, v) - vOrder + 1;
    const NurbsH3 P = NurbsEvaluate(uOrder, uKnot, iso.data(), uFirstCp, 1, u, dPdu);
    for (int i = 0; i < vOrder; ++i) iso[i] = NurbsEvaluate(uOrder, uKnot, cp + (size_t)(vFirstCp + i) * ucp, 0, 1, u, nullptr);
    (void)NurbsEvaluate(vOrder, vKnot, iso.data(), vFirstCp, 1, v, dPdv);
    (void)vcp;
    return V3(P.x / P.w, P.y / P.w, P.z / P.w);
}
// an intersectable shape after refinement
struct Isect {
    int kind;             // PBRTGPU_SHAPE_*
    TriMesh *mesh = nullptr;
    int tri = -1;
    Quadric *quad = nullptr;
    int inst = -1;        // PBRTGPU_SHAPE_INSTANCE: instance index
    BBox instBound;       // TransformedPrimitive::WorldBound (motion bounds)
    BBox WorldBound() const {
        if (kind == PBRTGPU_SHAPE_INSTANCE) return instBound;
        if (kind == PBRTGPU_SHAPE_TRIANGLE) {
            const V3 &p1 = mesh->p[mesh->vi[3 * tri]], &p2 = mesh->p[mesh->vi[3 * tri + 1]], &p3 = mesh->p[mesh->vi[3 * tri + 2]];
            return Union(BBox(p1, p2), p3);
        }
        return quad->o2w(quad->ObjectBound());
    }
    float Area() const {
        if (kind == PBRTGPU_SHAPE_TRIANGLE) {
            const V3 &p1 = mesh->p[mesh->vi[3 * tri]], &p2 = mesh->p[mesh->vi[3 * tri + 1]], &p3 = mesh->p[mesh->vi[3 * tri + 2]];
            return 0.5f * Length(Cross(p2 - p1, p3 - p1));
        }
        return quad->Area();
    }
};

// measured BRDF (measured.cpp:90-128): samples in BRDFRemap coordinates with spectra
struct BrdfSample { V3 p; Spec v; };
struct MeasuredData { std::vector<BrdfSample> samples; int flatFirst = -1; };
struct MaterialObj {
    pbrtgpu_material m{};
    std::vector<Spec> spectra;
    std::shared_ptr<MeasuredData> measured;
    int flatIndex = -1;
    uint32_t refId = 0;   // Material::materialId (material.h:39: constructor counter from 1)
};
struct LightObj {
    pbrtgpu_light l{};
    LightObj() { l.map_tex = -1; l.dist_off = -1; l.dist_nu = l.dist_nv = 1; }   // no decoded environment map
    Spec L;
    std::vector<Isect> shapeSet;      // area light ShapeSet (light.cpp:114-135)
};
struct PrimObj {
    std::shared_ptr<ShapeObj> shape;
    std::shared_ptr<MaterialObj> mtl;
    int areaLight = -1;
    int instance = -1;    // animated shape -> TransformedPrimitive (index into instanceObjs)
    uint32_t refId = 0;   // Primitive::primitiveId of the GeometricPrimitive / TransformedPrimitive
    std::string name;     // the Shape directive's name (api.cpp:1117 primitiveNames)
};

struct SDVertex { V3 P; int startFace = -1; int child = -1; bool regular = false, boundary = false; };
struct SDFace { int v[3] = {-1, -1, -1}; int f[3] = {-1, -1, -1}; int children[4] = {-1, -1, -1, -1}; };

struct ShapeObj {
    enum { MESH, QUADRIC, LOOP, HFIELD } kind;   // HFIELD: a Heightfield or NURBS, its refined TriangleMesh in mesh
    std::shared_ptr<TriMesh> mesh;
    std::shared_ptr<Quadric> quad;
    // loop subdivision control mesh
    Xform o2w;
    bool ro = false;
    int nLevels = 0;
    std::vector<SDVertex> verts;
    std::vector<SDFace> faces;
    std::shared_ptr<TriMesh> refined;   // cached LoopSubdiv::Refine result
};

#define NEXT(i) (((i) + 1) % 3)
#define PREV(i) (((i) + 2) % 3)

// ---------------------- Loop subdivision (loopsubdiv.cpp) ---------------------------
struct LoopMesh {
    std::vector<SDVertex> &V;
    std::vector<SDFace> &F;
    int vnum(int f, int v) const {
        for (int i = 0; i < 3; ++i) if (F[f].v[i] == v) return i;
        throw std::runtime_error("loopsubdiv: vnum logic error");
    }
    int nextFace(int f, int v) const { return F[f].f[vnum(f, v)]; }
    int prevFace(int f, int v) const { return F[f].f[PREV(vnum(f, v))]; }
    int nextVert(int f, int v) const { return F[f].v[NEXT(vnum(f, v))]; }
    int prevVert(int f, int v) const { return F[f].v[PREV(vnum(f, v))]; }
    int otherVert(int f, int v0, int v1) const {
        for (int i = 0; i < 3; ++i) if (F[f].v[i] != v0 && F[f].v[i] != v1) return F[f].v[i];
        throw std::runtime_error("loopsubdiv: otherVert logic error");
    }
    int valence(int v) const {   // loopsubdiv.cpp:121-143
        int f = V[v].startFace;
        if (!V[v].boundary) {
            int nf = 1;
            while ((f = nextFace(f, v)) != V[v].startFace) ++nf;
            return nf;
        }
        int nf = 1;
        while ((f = nextFace(f, v)) != -1) ++nf;
        f = V[v].startFace;
        while ((f = prevFace(f, v)) != -1) ++nf;
        return nf + 1;
    }
    void oneRing(int v, std::vector<V3> &P) const {   // loopsubdiv.cpp:451-470
        P.clear();
        if (!V[v].boundary) {
            int face = V[v].startFace;
            do { P.push_back(V[nextVert(face, v)].P); face = nextFace(face, v); } while (face != V[v].startFace);
        } else {
            int face = V[v].startFace, f2;
            while ((f2 = nextFace(face, v)) != -1) face = f2;
            P.push_back(V[nextVert(face, v)].P);
            do { P.push_back(V[prevVert(face, v)].P); face = prevFace(face, v); } while (face != -1);
        }
    }
    V3 weightOneRing(int v, float beta) const {   // loopsubdiv.cpp:440-449
        int valence_ = valence(v);
        std::vector<V3> Pring;
        oneRing(v, Pring);
        V3 P = (1 - valence_ * beta) * V[v].P;
        for (int i = 0; i < valence_; ++i) P += beta * Pring[i];
        return P;
    }
    V3 weightBoundary(int v, float beta) const {   // loopsubdiv.cpp:473-482
        int valence_ = valence(v);
        std::vector<V3> Pring;
        oneRing(v, Pring);
        V3 P = (1 - 2 * beta) * V[v].P;
        P += beta * Pring[0];
        P += beta * Pring[valence_ - 1];
        return P;
    }
};
static float LoopBeta(int valence) { return valence == 3 ? 3.f / 16.f : 3.f / (8.f * valence); }
static float LoopGamma(int valence) { return 1.f / (valence + 3.f / (8.f * LoopBeta(valence))); }

// LoopSubdiv constructor (loopsubdiv.cpp:147-198)
static void LoopInit(ShapeObj &s, int nfaces, int nvertices, const int *vi, const V3 *P) {
    s.verts.resize(nvertices);
    for (int i = 0; i < nvertices; ++i) s.verts[i] = SDVertex(), s.verts[i].P = P[i];
    s.faces.resize(nfaces);
    const int *vp = vi;
    for (int i = 0; i < nfaces; ++i) {
        for (int j = 0; j < 3; ++j) {
            int v = vp[j];
            s.faces[i].v[j] = v;
            s.verts[v].startFace = i;
        }
        vp += 3;
    }
    struct Edge { int f0; int f0edgeNum; };
    std::map<std::pair<int, int>, Edge> edges;
    for (int i = 0; i < nfaces; ++i) {
        for (int edgeNum = 0; edgeNum < 3; ++edgeNum) {
            int a = s.faces[i].v[edgeNum], b = s.faces[i].v[NEXT(edgeNum)];
            std::pair<int, int> key(std::min(a, b), std::max(a, b));
            auto it = edges.find(key);
            if (it == edges.end()) edges[key] = Edge{i, edgeNum};
            else {
                Edge e = it->second;
                s.faces[e.f0].f[e.f0edgeNum] = i;
                s.faces[i].f[edgeNum] = e.f0;
                edges.erase(it);
            }
        }
    }
    LoopMesh lm{s.verts, s.faces};
    for (int i = 0; i < nvertices; ++i) {
        int f = s.verts[i].startFace;
        do { f = lm.nextFace(f, i); } while (f != -1 && f != s.verts[i].startFace);
        s.verts[i].boundary = (f == -1);
        if (!s.verts[i].boundary && lm.valence(i) == 6) s.verts[i].regular = true;
        else if (s.verts[i].boundary && lm.valence(i) == 4) s.verts[i].regular = true;
        else s.verts[i].regular = false;
    }
}

// LoopSubdiv::Refine (loopsubdiv.cpp:222-437): limit positions (object space), limit normals
// and the refined faces' vertex indices
static void LoopRefineCore(ShapeObj &s, std::vector<V3> &Plimit, std::vector<V3> &Ns, std::vector<int> &vi) {
    std::vector<SDVertex> V = s.verts;
    std::vector<SDFace> F = s.faces;
    std::vector<int> f(F.size()), v(V.size());
    for (size_t i = 0; i < F.size(); ++i) f[i] = (int)i;
    for (size_t i = 0; i < V.size(); ++i) v[i] = (int)i;
    LoopMesh lm{V, F};
    for (int level = 0; level < s.nLevels; ++level) {
        std::vector<int> newFaces, newVertices;
        for (size_t j = 0; j < v.size(); ++j) {
            SDVertex c; c.regular = V[v[j]].regular; c.boundary = V[v[j]].boundary;
            V.push_back(c);
            V[v[j]].child = (int)V.size() - 1;
            newVertices.push_back((int)V.size() - 1);
        }
        for (size_t j = 0; j < f.size(); ++j)
            for (int k = 0; k < 4; ++k) {
                F.push_back(SDFace());
                F[f[j]].children[k] = (int)F.size() - 1;
                newFaces.push_back((int)F.size() - 1);
            }
        // even vertices
        for (size_t j = 0; j < v.size(); ++j) {
            int vv = v[j];
            V3 P;
            if (!V[vv].boundary) {
                if (V[vv].regular) P = lm.weightOneRing(vv, 1.f / 16.f);
                else P = lm.weightOneRing(vv, LoopBeta(lm.valence(vv)));
            } else P = lm.weightBoundary(vv, 1.f / 8.f);
            V[V[vv].child].P = P;
        }
        // odd (edge) vertices
        std::map<std::pair<int, int>, int> edgeVerts;
        for (size_t j = 0; j < f.size(); ++j) {
            int face = f[j];
            for (int k = 0; k < 3; ++k) {
                int e0 = F[face].v[k], e1 = F[face].v[NEXT(k)];
                std::pair<int, int> key(std::min(e0, e1), std::max(e0, e1));
                auto it = edgeVerts.find(key);
                if (it == edgeVerts.end()) {
                    SDVertex nv;
                    nv.regular = true;
                    nv.boundary = (F[face].f[k] == -1);
                    nv.startFace = F[face].children[3];
                    int a = key.first, b = key.second;
                    if (nv.boundary) {
                        nv.P = 0.5f * V[a].P;
                        nv.P += 0.5f * V[b].P;
                    } else {
                        nv.P = 3.f / 8.f * V[a].P;
                        nv.P += 3.f / 8.f * V[b].P;
                        nv.P += 1.f / 8.f * V[lm.otherVert(face, a, b)].P;
                        nv.P += 1.f / 8.f * V[lm.otherVert(F[face].f[k], a, b)].P;
                    }
                    V.push_back(nv);
                    newVertices.push_back((int)V.size() - 1);
                    edgeVerts[key] = (int)V.size() - 1;
                }
            }
        }
        // topology: even vertex start faces
        for (size_t j = 0; j < v.size(); ++j) {
            int vert = v[j];
            int vertNum = lm.vnum(V[vert].startFace, vert);
            V[V[vert].child].startFace = F[V[vert].startFace].children[vertNum];
        }
        // face neighbour pointers
        for (size_t j = 0; j < f.size(); ++j) {
            int face = f[j];
            for (int k = 0; k < 3; ++k) {
                F[F[face].children[3]].f[k] = F[face].children[NEXT(k)];
                F[F[face].children[k]].f[NEXT(k)] = F[face].children[3];
                int f2 = F[face].f[k];
                F[F[face].children[k]].f[k] = f2 != -1 ? F[f2].children[lm.vnum(f2, F[face].v[k])] : -1;
                f2 = F[face].f[PREV(k)];
                F[F[face].children[k]].f[PREV(k)] = f2 != -1 ? F[f2].children[lm.vnum(f2, F[face].v[k])] : -1;
            }
        }
        // face vertex pointers
        for (size_t j = 0; j < f.size(); ++j) {
            int face = f[j];
            for (int k = 0; k < 3; ++k) {
                F[F[face].children[k]].v[k] = V[F[face].v[k]].child;
                int e0 = F[face].v[k], e1 = F[face].v[NEXT(k)];
                int vert = edgeVerts[std::make_pair(std::min(e0, e1), std::max(e0, e1))];
                F[F[face].children[k]].v[NEXT(k)] = vert;
                F[F[face].children[NEXT(k)]].v[k] = vert;
                F[F[face].children[3]].v[k] = vert;
            }
        }
        f = newFaces;
        v = newVertices;
    }
    // limit surface
    Plimit.assign(v.size(), V3());
    for (size_t i = 0; i < v.size(); ++i) {
        if (V[v[i]].boundary) Plimit[i] = lm.weightBoundary(v[i], 1.f / 5.f);
        else Plimit[i] = lm.weightOneRing(v[i], LoopGamma(lm.valence(v[i])));
    }
    for (size_t i = 0; i < v.size(); ++i) V[v[i]].P = Plimit[i];
    // tangents -> normals
    Ns.clear();
    Ns.reserve(v.size());
    std::vector<V3> Pring;
    for (size_t i = 0; i < v.size(); ++i) {
        int vert = v[i];
        V3 S(0, 0, 0), T(0, 0, 0);
        int valence = lm.valence(vert);
        lm.oneRing(vert, Pring);
        if (!V[vert].boundary) {
            for (int k = 0; k < valence; ++k) {
                S += cosf(2.f * kPi * k / valence) * Pring[k];
                T += sinf(2.f * kPi * k / valence) * Pring[k];
            }
        } else {
            S = Pring[valence - 1] - Pring[0];
            if (valence == 2) T = (Pring[0] + Pring[1]) - 2 * V[vert].P;
            else if (valence == 3) T = Pring[1] - V[vert].P;
            else if (valence == 4)
                T = -1 * Pring[0] + 2 * Pring[1] + 2 * Pring[2] + -1 * Pring[3] + -2 * V[vert].P;
            else {
                float theta = kPi / float(valence - 1);
                T = sinf(theta) * (Pring[0] + Pring[valence - 1]);
                for (int k = 1; k < valence - 1; ++k) {
                    float wt = (2 * cosf(theta) - 2) * sinf((k) * theta);
                    T += wt * Pring[k];
                }
                T = -T;
            }
        }
        Ns.push_back(Cross(S, T));
    }
    std::map<int, int> used;
    for (size_t i = 0; i < v.size(); ++i) used[v[i]] = (int)i;
    vi.clear();
    for (size_t i = 0; i < f.size(); ++i)
        for (int j = 0; j < 3; ++j) vi.push_back(used[F[f[i]].v[j]]);
}

// the refinement of a loopsubdiv shape: on the GPU when a subdivider is set
// (pbrthost_set_loop_subdivider; pbrtgpu_loop_subdivide_hook), else LoopRefineCore
static pbrthost_loop_subdivider g_loopFn = nullptr;
static void *g_loopUser = nullptr;
static std::shared_ptr<TriMesh> LoopRefine(ShapeObj &s) {
    std::vector<V3> Plimit, Ns;
    std::vector<int> vi;
    if (g_loopFn) {
        const int nf = (int)s.faces.size(), nv = (int)s.verts.size();
        std::vector<int> cvi(3 * (size_t)nf);
        std::vector<float> cP(3 * (size_t)nv);
        for (int i = 0; i < nf; ++i)
            for (int j = 0; j < 3; ++j) cvi[3 * i + j] = s.faces[i].v[j];
        for (int i = 0; i < nv; ++i) { cP[3 * i] = s.verts[i].P.x; cP[3 * i + 1] = s.verts[i].P.y; cP[3 * i + 2] = s.verts[i].P.z; }
        int nvOut = 0;
        if (g_loopFn(g_loopUser, nf, nv, cvi.data(), cP.data(), s.nLevels, &nvOut, nullptr, nullptr, nullptr) != 0)
            throw std::runtime_error("loopsubdiv: the GPU subdivider failed (sizes)");
        const size_t nfOut = (size_t)nf << (2 * s.nLevels);
        std::vector<float> P(3 * (size_t)nvOut), N(3 * (size_t)nvOut);
        vi.resize(3 * nfOut);
        if (g_loopFn(g_loopUser, nf, nv, cvi.data(), cP.data(), s.nLevels, &nvOut, P.data(), N.data(), vi.data()) != 0)
            throw std::runtime_error("loopsubdiv: the GPU subdivider failed");
        Plimit.resize(nvOut);
        Ns.resize(nvOut);
        for (int i = 0; i < nvOut; ++i) {
            Plimit[i] = V3(P[3 * i], P[3 * i + 1], P[3 * i + 2]);
            Ns[i] = V3(N[3 * i], N[3 * i + 1], N[3 * i + 2]);
        }
    } else LoopRefineCore(s, Plimit, Ns, vi);
    auto mesh = std::make_shared<TriMesh>();
    mesh->o2w = s.o2w;
    mesh->ro = s.ro;
    mesh->swaps = s.o2w.SwapsHandedness();
    mesh->ntris = (int)vi.size() / 3;
    mesh->nverts = (int)Plimit.size();
    mesh->vi = vi;
    mesh->p.resize(Plimit.size());
    for (size_t i = 0; i < Plimit.size(); ++i) mesh->p[i] = s.o2w.Point(Plimit[i]);
    mesh->n = Ns;
    return mesh;
}

extern "C" int pbrthost_set_loop_subdivider(pbrthost_loop_subdivider fn, void *user) {
    g_loopFn = fn;
    g_loopUser = user;
    return 0;
}

// the host refinement of a control mesh (object space), for tests of the GPU subdivider
extern "C" int pbrthost_loop_refine(int32_t nf, int32_t nv, const int32_t *vi, const float *P, int32_t levels,
                                    int32_t *nv_out, float *P_out, float *N_out, int32_t *vi_out) {
    try {
        if (nf < 1 || nv < 1 || levels < 0 || !vi || !P || !nv_out) return -1;
        std::vector<V3> cp(nv);
        for (int i = 0; i < nv; ++i) cp[i] = V3(P[3 * i], P[3 * i + 1], P[3 * i + 2]);
        ShapeObj s;
        s.kind = ShapeObj::LOOP;
        s.nLevels = levels;
        LoopInit(s, nf, nv, vi, cp.data());
        std::vector<V3> Pl, Ns;
        std::vector<int> fvi;
        LoopRefineCore(s, Pl, Ns, fvi);
        *nv_out = (int32_t)Pl.size();
        if (P_out) {
            for (size_t i = 0; i < Pl.size(); ++i) {
                P_out[3 * i] = Pl[i].x; P_out[3 * i + 1] = Pl[i].y; P_out[3 * i + 2] = Pl[i].z;
                N_out[3 * i] = Ns[i].x; N_out[3 * i + 1] = Ns[i].y; N_out[3 * i + 2] = Ns[i].z;
            }
            std::copy(fvi.begin(), fvi.end(), vi_out);
        }
        return 0;
    } catch (const std::exception &) {
        return -1;
    }
}

// ------------------------------------------------------------------------------------
// Image maps: ReadImage for the formats this build reads without OpenEXR (imageio.cpp:45-66),
// the decoders' texel values (RGBSpectrum, 3 floats per texel) and MIPMap construction
// (mipmap.h:119-193).  Float expressions in the reference's operand order.
// ------------------------------------------------------------------------------------
// ReadImageTGA (imageio.cpp:443-533): uncompressed true colour (24 / 32 bit) and 8-bit grey;
// the 18-byte header is followed directly by the pixels (the ID field is not skipped); texels in
// the file's row order, then the origin bits' horizontal / vertical flips.  false: the reference
// returns NULL (Error)
static bool ReadTGA(const std::string &fn, std::vector<float> &rgb, int *w, int *h) {
    FILE *f = fopen(fn.c_str(), "rb");
    if (!f) return false;
    unsigned char hd[18] = {0};
    const size_t nh = fread(hd, 1, 18, f);
    (void)nh;   // the reference reads its fields with unchecked fread calls
    auto s16 = [&](int o) { return (int)(int16_t)(uint16_t)(hd[o] | (hd[o + 1] << 8)); };
    const int imageType = hd[2], width = s16(12), height = s16(14), depth = hd[16], attr = hd[17];
    if (((attr & 0xf) != 8 && (attr & 0xf) != 0) || (attr & 0xc0) != 0 ||
        (imageType == 2 && depth != 32 && depth != 24) || (imageType == 3 && depth != 8) ||
        (imageType != 2 && imageType != 3) || width <= 0 || height <= 0) {
        fclose(f);
        return false;
    }
    const int pixbytes = depth == 32 ? 4 : (depth == 24 ? 3 : 1);
    const size_t size = (size_t)width * height * pixbytes;
    std::vector<unsigned char> src(size);
    const bool got = fread(src.data(), 1, size, f) == size;
    fclose(f);
    if (!got) return false;   // "Premature end-of-file"
    rgb.assign((size_t)width * height * 3, 0.f);
    const unsigned char *p = src.data();
    for (size_t i = 0; i < (size_t)width * height; ++i) {
        if (pixbytes == 1) {
            const float v = (*p++) / 255.f;
            rgb[3 * i] = rgb[3 * i + 1] = rgb[3 * i + 2] = v;   // RGBSpectrum(v)
        } else {
            const float b = (*p++) / 255.f, g = (*p++) / 255.f, r = (*p++) / 255.f;
            rgb[3 * i] = r; rgb[3 * i + 1] = g; rgb[3 * i + 2] = b;   // FromRGB(c)
            if (pixbytes == 4) ++p;
        }
    }
    auto swapTexel = [&](size_t a, size_t b) { for (int k = 0; k < 3; ++k) std::swap(rgb[3 * a + k], rgb[3 * b + k]); };
    if (attr & 0x10)
        for (int y = 0; y < height; ++y)
            for (int x = 0; x < width / 2; ++x) swapTexel((size_t)y * width + x, (size_t)y * width + (width - 1 - x));
    if (attr & 0x20)
        for (int y = 0; y < height / 2; ++y)
            for (int x = 0; x < width; ++x) swapTexel((size_t)y * width + x, (size_t)(height - 1 - y) * width + x);
    *w = width; *h = height;
    return true;
}
// ReadImagePFM (imageio.cpp:574-650): "Pf" (grey) / "PF" (RGB) header words split at ' ', '\n'
// and '\t', |scale| != 1 multiplies, its sign gives the byte order; no vertical flip
static bool ReadPFM(const std::string &fn, std::vector<float> &rgb, int *w, int *h) {
    FILE *f = fopen(fn.c_str(), "rb");
    if (!f) return false;
    auto word = [&](std::string &s) -> bool {   // readWord: up to 80 characters before whitespace
        s.clear();
        int c = fgetc(f);
        while (c != EOF && (char)c != ' ' && (char)c != '\n' && (char)c != '\t' && s.size() < 80) {
            s.push_back((char)c);
            c = fgetc(f);
        }
        return s.size() < 80;
    };
    std::string tok;
    int nc = 0;
    bool ok = word(tok);
    if (ok) nc = tok == "Pf" ? 1 : (tok == "PF" ? 3 : 0);
    ok = ok && nc > 0;
    int width = 0, height = 0;
    float scale = 0.f;
    ok = ok && word(tok);
    if (ok) width = atoi(tok.c_str());
    ok = ok && word(tok);
    if (ok) height = atoi(tok.c_str());
    ok = ok && word(tok);
    if (ok) sscanf(tok.c_str(), "%f", &scale);
    ok = ok && width > 0 && height > 0;
    std::vector<float> data;
    if (ok) {
        data.resize((size_t)nc * width * height);
        ok = fread(data.data(), sizeof(float), data.size(), f) == data.size();
    }
    fclose(f);
    if (!ok) return false;
    if (!(scale < 0.f))   // big-endian file on this little-endian host
        for (float &v : data) {
            uint8_t b[4];
            memcpy(b, &v, 4);
            std::swap(b[0], b[3]); std::swap(b[1], b[2]);
            memcpy(&v, b, 4);
        }
    if (fabsf(scale) != 1.f)
        for (float &v : data) v *= fabsf(scale);
    rgb.assign((size_t)width * height * 3, 0.f);
    for (size_t i = 0; i < (size_t)width * height; ++i)
        for (int k = 0; k < 3; ++k) rgb[3 * i + k] = nc == 1 ? data[i] : data[3 * i + k];
    *w = width; *h = height;
    return true;
}
static float Lanczos(float x, float tau = 2.f) {   // texture.cpp:258-266 (M_PI a float literal, pbrt.h:179)
    x = fabsf(x);
    if (x < 1e-5) return 1;
    if (x > 1.) return 0;
    x *= 3.14159265358979323846f;
    float s = sinf(x * tau) / (x * tau);
    float lanczos = sinf(x) / x;
    return s * lanczos;
}
static int ModI(int a, int b) { int n = int(a / b); a -= n * b; if (a < 0) a += b; return a; }   // pbrt.h Mod
static float Log2f(float x) { static float invLog2 = 1.f / logf(2.f); return logf(x) * invLog2; }   // pbrt.h:243-246
// MIPMap<T>(sres, tres, img, ..., wrapMode) (mipmap.h:119-193) for NC floats per texel (3: the
// RGBSpectrum of a spectrum texture, 1: a float texture): every pyramid level appended to `out`,
// level 0 first; returns (width, height, nLevels)
static void BuildMipmap(int sres, int tres, std::vector<float> img, int nc, int wrap, std::vector<float> &out, int *W,
                        int *H, int *levels) {
    auto isPow2 = [](int v) { return (v & (v - 1)) == 0; };
    auto roundUpPow2 = [](uint32_t v) { v--; v |= v >> 1; v |= v >> 2; v |= v >> 4; v |= v >> 8; v |= v >> 16; return v + 1; };
    struct RW { int first; float w[4]; };
    auto weights = [&](uint32_t oldres, uint32_t newres) {   // resampleWeights (mipmap.h:75-96)
        std::vector<RW> wt(newres);
        const float filterwidth = 2.f;
        for (uint32_t i = 0; i < newres; ++i) {
            float center = (i + .5f) * oldres / newres;
            wt[i].first = (int)floorf((center - filterwidth) + 0.5f);
            for (int j = 0; j < 4; ++j) {
                float pos = wt[i].first + j + .5f;
                wt[i].w[j] = Lanczos((pos - center) / filterwidth);
            }
            float invSumWts = 1.f / (wt[i].w[0] + wt[i].w[1] + wt[i].w[2] + wt[i].w[3]);
            for (int j = 0; j < 4; ++j) wt[i].w[j] *= invSumWts;
        }
        return wt;
    };
    auto wrapIdx = [&](int v, int n) {
        if (wrap == PBRTGPU_WRAP_REPEAT) return ModI(v, n);
        if (wrap == PBRTGPU_WRAP_CLAMP) return v < 0 ? 0 : (v > n - 1 ? n - 1 : v);
        return v;
    };
    if (!isPow2(sres) || !isPow2(tres)) {
        const uint32_t sPow2 = roundUpPow2((uint32_t)sres), tPow2 = roundUpPow2((uint32_t)tres);
        std::vector<float> res((size_t)sPow2 * tPow2 * nc, 0.f);
        const std::vector<RW> sw = weights((uint32_t)sres, sPow2);
        for (int t = 0; t < tres; ++t)
            for (uint32_t s = 0; s < sPow2; ++s) {
                float *o = &res[((size_t)t * sPow2 + s) * nc];
                for (int k = 0; k < nc; ++k) o[k] = 0.f;
                for (int j = 0; j < 4; ++j) {
                    const int origS = wrapIdx(sw[s].first + j, sres);
                    if (origS >= 0 && origS < sres)
                        for (int k = 0; k < nc; ++k) o[k] += img[((size_t)t * sres + origS) * nc + k] * sw[s].w[j];
                }
            }
        const std::vector<RW> tw = weights((uint32_t)tres, tPow2);
        std::vector<float> work((size_t)tPow2 * nc);
        for (uint32_t s = 0; s < sPow2; ++s) {
            for (uint32_t t = 0; t < tPow2; ++t) {
                float *o = &work[(size_t)t * nc];
                for (int k = 0; k < nc; ++k) o[k] = 0.f;
                for (int j = 0; j < 4; ++j) {
                    const int off = wrapIdx(tw[t].first + j, tres);
                    if (off >= 0 && off < tres)
                        for (int k = 0; k < nc; ++k) o[k] += res[((size_t)off * sPow2 + s) * nc + k] * tw[t].w[j];
                }
            }
            for (uint32_t t = 0; t < tPow2; ++t)
                for (int k = 0; k < nc; ++k) {   // clamp(v): Clamp(v, 0, INFINITY)
                    const float v = work[(size_t)t * nc + k];
                    res[((size_t)t * sPow2 + s) * nc + k] = v < 0.f ? 0.f : (v > INFINITY ? INFINITY : v);
                }
        }
        img.swap(res);
        sres = (int)sPow2;
        tres = (int)tPow2;
    }
    const int nLevels = 1 + (int)floorf(Log2f(float(std::max(sres, tres))));   // 1 + Log2Int
    const size_t base = out.size();
    out.insert(out.end(), img.begin(), img.end());
    size_t prev = base;
    int pw = sres, ph = tres;
    for (int i = 1; i < nLevels; ++i) {
        const int sR = std::max(1, pw / 2), tR = std::max(1, ph / 2);
        const size_t cur = out.size();
        out.resize(cur + (size_t)sR * tR * nc);
        auto texel = [&](int s, int t, int k) -> float {   // Texel(i - 1, s, t) with the wrap mode
            if (wrap == PBRTGPU_WRAP_REPEAT) { s = ModI(s, pw); t = ModI(t, ph); }
            else if (wrap == PBRTGPU_WRAP_CLAMP) { s = s < 0 ? 0 : (s > pw - 1 ? pw - 1 : s); t = t < 0 ? 0 : (t > ph - 1 ? ph - 1 : t); }
            else if (s < 0 || s >= pw || t < 0 || t >= ph) return 0.f;
            return out[prev + ((size_t)t * pw + s) * nc + k];
        };
        for (int t = 0; t < tR; ++t)
            for (int s = 0; s < sR; ++s)
                for (int k = 0; k < nc; ++k)
                    out[cur + ((size_t)t * sR + s) * nc + k] =
                        .25f * (texel(2 * s, 2 * t, k) + texel(2 * s + 1, 2 * t, k) + texel(2 * s, 2 * t + 1, k) +
                                texel(2 * s + 1, 2 * t + 1, k));
        prev = cur;
        pw = sR;
        ph = tR;
    }
    *W = sres; *H = tres; *levels = nLevels;
}

class Builder {
public:
    Builder(const std::string &path, const RenderOverrides &ov, HostScene *out)
        : ov(ov), out(out), spec(ov.bands, ov.bands == 30 ? 400 : 395, ov.bands == 30 ? 700 : 715) {
        size_t sl = path.find_last_of('/');
        searchDir = sl == std::string::npos ? std::string(".") : path.substr(0, sl);
    }
    void Run(const std::string &path) {
        tLoad0 = std::chrono::steady_clock::now();
        if (!lex.Open(path)) throw std::runtime_error("cannot open scene file " + path);
        Parse();
        if (!worldEnded) throw std::runtime_error("scene has no WorldEnd");
    }

private:
    static const int MAXT = 2;
    struct TransformSet {
        Xform t[MAXT];
        bool IsAnimated() const { return t[0] != t[1]; }
    };
    struct GState {
        std::map<std::string, FloatTex> floatTextures;
        std::map<std::string, SpecTex> spectrumTextures;
        ParamSet materialParams;
        std::string material = "matte";
        std::map<std::string, std::shared_ptr<MaterialObj> > namedMaterials;
        std::string currentNamedMaterial;
        ParamSet areaLightParams;
        std::string areaLight;
        bool reverseOrientation = false;
    };

    RenderOverrides ov;
    HostScene *out;
    std::chrono::steady_clock::time_point tLoad0;
    SpectrumCtx spec;
    Lexer lex;
    std::string searchDir;
    bool worldEnded = false;
    Token tok;
    bool havePeek = false;

    TransformSet curT;
    int activeBits = 3;
    std::map<std::string, TransformSet> namedCS;
    GState gs;
    std::vector<GState> pushedGS;
    std::vector<TransformSet> pushedT;
    std::vector<int> pushedBits;
    std::map<Xform, std::pair<Xform, Xform> > tcache;   // key compares m only (first wins)
    float tStart = 0.f, tEnd = 1.f;
    ParamSet filmParams, cameraParams, samplerParams, surfParams, accelParams;
    std::string surfName = "directlighting";   // RenderOptions::SurfIntegratorName default (api.cpp:222)
    std::string rendererName = "sampler";      // RenderOptions::RendererName default (api.cpp:225)
    ParamSet rendererParams;
    std::string cameraName = "perspective";
    TransformSet cameraToWorld;
    std::vector<std::shared_ptr<LightObj> > lights;
    std::vector<PrimObj> primitives;
    // Primitive / Material constructor counters (primitive.cpp:32, material.cpp:34): the ids
    // the MetadataIntegrator reports, replayed in the reference's construction order
    uint32_t nextPrimId = 1, nextMatId = 1;
    std::vector<std::shared_ptr<TriMesh> > allMeshes;
    std::vector<std::shared_ptr<Quadric> > allQuads;

    // ----------------------------- tokens -----------------------------------------
    bool Peek(Token *t) {
        if (!havePeek) { lex.Next(&tok); havePeek = true; }
        *t = tok;
        return tok.kind != Token::END;
    }
    Token Take() { Token t; Peek(&t); havePeek = false; return t; }
    float Num() {
        Token t = Take();
        if (t.kind != Token::NUMBER) throw std::runtime_error("expected number, got '" + t.text + "'");
        return t.num;
    }
    std::string Str() {
        Token t = Take();
        if (t.kind != Token::STRING) throw std::runtime_error("expected string, got '" + t.text + "'");
        return t.text;
    }
    void NumArray(float *v, int n) {
        Token t; Peek(&t);
        bool br = t.kind == Token::LBRACK;
        if (br) Take();
        for (int i = 0; i < n; ++i) v[i] = Num();
        if (br) { Token e = Take(); if (e.kind != Token::RBRACK) throw std::runtime_error("expected ]"); }
    }
    std::string Resolve(const std::string &fn) const {
        if (fn.empty() || fn[0] == '/') return fn;
        return searchDir + "/" + fn;
    }
    ParamSet Params() {   // pbrtparse.yy paramlist + InitParamSet (pbrtparse.yy:620-760)
        ParamSet ps;
        for (;;) {
            Token t;
            if (!Peek(&t) || t.kind != Token::STRING) break;
            std::string decl = Take().text;
            // value: single or bracketed list of numbers or strings
            std::vector<float> nums;
            std::vector<std::string> strs;
            Token v = Take();
            if (v.kind == Token::LBRACK) {
                for (;;) {
                    Token e = Take();
                    if (e.kind == Token::RBRACK) break;
                    if (e.kind == Token::NUMBER) nums.push_back(e.num);
                    else if (e.kind == Token::STRING) strs.push_back(e.text);
                    else throw std::runtime_error("bad parameter list for " + decl);
                }
            } else if (v.kind == Token::NUMBER) nums.push_back(v.num);
            else if (v.kind == Token::STRING) strs.push_back(v.text);
            else throw std::runtime_error("bad parameter value for " + decl);
            AddParam(ps, decl, nums, strs);
        }
        return ps;
    }
    void AddParam(ParamSet &ps, const std::string &decl, const std::vector<float> &nums,
                  const std::vector<std::string> &strs) {
        size_t a = 0;
        while (a < decl.size() && isspace((unsigned char)decl[a])) ++a;
        static const char *types[] = {"float", "integer", "bool", "point", "vector", "normal", "string",
                                      "texture", "color", "rgb", "xyz", "blackbody", "spectrum"};
        int type = -1;
        for (int k = 0; k < 13; ++k)
            if (decl.compare(a, strlen(types[k]), types[k]) == 0) { type = k; a += strlen(types[k]); break; }
        if (type < 0) { out->warnings.push_back("unknown parameter type: " + decl); return; }
        while (a < decl.size() && isspace((unsigned char)decl[a])) ++a;
        size_t e = a;
        while (e < decl.size() && !isspace((unsigned char)decl[e])) ++e;
        Param p;
        p.name = decl.substr(a, e - a);
        switch (type) {
            case 0: p.cat = P_FLOAT; p.f = nums; break;
            case 1: p.cat = P_INT; for (float x : nums) p.i.push_back(int(x)); break;
            case 2: p.cat = P_BOOL; for (auto &s : strs) p.b.push_back(s == "true"); break;
            case 3: p.cat = P_POINT; p.f.assign(nums.begin(), nums.begin() + (nums.size() / 3) * 3); break;
            case 4: p.cat = P_VECTOR; p.f.assign(nums.begin(), nums.begin() + (nums.size() / 3) * 3); break;
            case 5: p.cat = P_NORMAL; p.f.assign(nums.begin(), nums.begin() + (nums.size() / 3) * 3); break;
            case 6: p.cat = P_STRING; p.s = strs; break;
            case 7: p.cat = P_TEXTURE; p.s = strs; break;
            case 8: case 9:   // AddRGBSpectrum: FromRGB (reflectance) for every colour parameter
                p.cat = P_SPECTRUM;
                for (size_t k = 0; k + 2 < nums.size(); k += 3) p.spec.push_back(spec.FromRGB(&nums[k]));
                break;
            case 10:
                p.cat = P_SPECTRUM;
                for (size_t k = 0; k + 2 < nums.size(); k += 3) p.spec.push_back(spec.FromXYZ(&nums[k]));
                break;
            case 11:
                p.cat = P_SPECTRUM;
                for (size_t k = 0; k + 1 < nums.size(); k += 2) p.spec.push_back(spec.Blackbody(nums[k], nums[k + 1]));
                break;
            case 12:
                p.cat = P_SPECTRUM;
                if (!strs.empty()) {
                    for (auto &fn : strs) p.spec.push_back(ReadSPD(Resolve(fn)));
                } else {
                    std::vector<float> wl, vv;
                    for (size_t k = 0; k + 1 < nums.size(); k += 2) { wl.push_back(nums[k]); vv.push_back(nums[k + 1]); }
                    p.spec.push_back(spec.FromSampled(wl.data(), vv.data(), (int)wl.size()));
                }
                break;
        }
        ps.Add(p);
    }
    Spec ReadSPD(const std::string &fn) {   // floatfile.cpp ReadFloatFile + paramset.cpp:145-178
        FILE *f = fopen(fn.c_str(), "r");
        if (!f) { out->warnings.push_back("unable to read SPD file " + fn + "; using black"); return spec.Const(0.f); }
        std::vector<float> vals;
        int c; bool inNumber = false; char buf[64]; int pos = 0;
        while ((c = getc(f)) != EOF) {
            if (c == '#') { while ((c = getc(f)) != EOF && c != '\n' && c != '\r') {} continue; }
            if (inNumber) {
                if (isdigit(c) || c == '.' || c == 'e' || c == '-' || c == '+') buf[pos++] = (char)c;
                else { buf[pos] = 0; vals.push_back((float)atof(buf)); inNumber = false; pos = 0; }
            } else if (isdigit(c) || c == '.' || c == '-' || c == '+') { inNumber = true; buf[pos++] = (char)c; }
            if (pos >= 63) pos = 62;
        }
        if (inNumber) { buf[pos] = 0; vals.push_back((float)atof(buf)); }
        fclose(f);
        std::vector<float> wl, v;
        for (size_t j = 0; j < vals.size() / 2; ++j) { wl.push_back(vals[2 * j]); v.push_back(vals[2 * j + 1]); }
        return spec.FromSampled(wl.data(), v.data(), (int)wl.size());
    }

    // ------------------------------ directives ------------------------------------
    void ForActive(const std::function<void(Xform &)> &fn) {
        for (int i = 0; i < MAXT; ++i) if (activeBits & (1 << i)) fn(curT.t[i]);
    }
    void Parse() {
        for (;;) {
            Token t = Take();
            if (t.kind == Token::END) return;
            if (t.kind != Token::IDENT) throw std::runtime_error("expected directive, got '" + t.text + "'");
            const std::string &d = t.text;
            if (d == "Identity") ForActive([](Xform &x) { x = Xform(); });
            else if (d == "Translate") { float v[3]; NumArray(v, 3); ForActive([&](Xform &x) { x = x * Translate(V3(v[0], v[1], v[2])); }); }
            else if (d == "Scale") { float v[3]; NumArray(v, 3); ForActive([&](Xform &x) { x = x * Scale(v[0], v[1], v[2]); }); }
            else if (d == "Rotate") { float v[4]; NumArray(v, 4); ForActive([&](Xform &x) { x = x * Rotate(v[0], V3(v[1], v[2], v[3])); }); }
            else if (d == "LookAt") {
                float v[9]; NumArray(v, 9);
                ForActive([&](Xform &x) { x = x * LookAt(V3(v[0], v[1], v[2]), V3(v[3], v[4], v[5]), V3(v[6], v[7], v[8])); });
            } else if (d == "ConcatTransform" || d == "Transform") {
                float tr[16]; NumArray(tr, 16);
                M4 m(tr[0], tr[4], tr[8], tr[12], tr[1], tr[5], tr[9], tr[13], tr[2], tr[6], tr[10], tr[14], tr[3], tr[7], tr[11], tr[15]);
                bool concat = d == "ConcatTransform";
                ForActive([&](Xform &x) { x = concat ? x * Xform(m) : Xform(m); });
            } else if (d == "CoordinateSystem") namedCS[Str()] = curT;
            else if (d == "CoordSysTransform") { std::string n = Str(); if (namedCS.count(n)) curT = namedCS[n]; }
            else if (d == "ActiveTransform") {
                Token a = Take();
                if (a.text == "All") activeBits = 3; else if (a.text == "EndTime") activeBits = 2; else if (a.text == "StartTime") activeBits = 1;
                else throw std::runtime_error("bad ActiveTransform " + a.text);
            } else if (d == "TransformTimes") { tStart = Num(); tEnd = Num(); }
            else if (d == "PixelFilter") {
                // api.cpp:857-860 keeps the name and parameters, MakeFilter (api.cpp:673-690) creates
                // the filter; the core renders the box filter at its default width (box.cpp:36-41),
                // the packaged scenes' only filter: anything else is refused, not approximated
                const std::string fname = Str();
                const ParamSet fp = Params();
                if (fname != "box" || fp.FindOneFloat("xwidth", .5f) != .5f || fp.FindOneFloat("ywidth", .5f) != .5f)
                    throw std::runtime_error("PixelFilter \"" + fname + "\": only the box filter of width .5 is supported");
            }
            else if (d == "Film") { Str(); filmParams = Params(); }
            else if (d == "Sampler") { Str(); samplerParams = Params(); }
            else if (d == "Accelerator") { Str(); accelParams = Params(); }
            else if (d == "SurfaceIntegrator") { surfName = Str(); surfParams = Params(); }
            else if (d == "VolumeIntegrator") { Str(); Params(); }
            else if (d == "Renderer") { rendererName = Str(); rendererParams = Params(); }
            else if (d == "Camera") {
                cameraName = Str(); cameraParams = Params();
                for (int i = 0; i < MAXT; ++i) cameraToWorld.t[i] = Inverse(curT.t[i]);
                namedCS["camera"] = cameraToWorld;
            } else if (d == "WorldBegin") {
                for (int i = 0; i < MAXT; ++i) curT.t[i] = Xform();
                activeBits = 3;
                namedCS["world"] = curT;
            } else if (d == "AttributeBegin") { pushedGS.push_back(gs); pushedT.push_back(curT); pushedBits.push_back(activeBits); }
            else if (d == "AttributeEnd") {
                if (pushedGS.empty()) { out->warnings.push_back("unmatched AttributeEnd"); continue; }
                gs = pushedGS.back(); pushedGS.pop_back();
                curT = pushedT.back(); pushedT.pop_back();
                activeBits = pushedBits.back(); pushedBits.pop_back();
            } else if (d == "TransformBegin") { pushedT.push_back(curT); pushedBits.push_back(activeBits); }
            else if (d == "TransformEnd") {
                if (pushedT.empty()) continue;
                curT = pushedT.back(); pushedT.pop_back();
                activeBits = pushedBits.back(); pushedBits.pop_back();
            } else if (d == "ReverseOrientation") gs.reverseOrientation = !gs.reverseOrientation;
            else if (d == "Material") { gs.material = Str(); gs.materialParams = Params(); gs.currentNamedMaterial = ""; }
            else if (d == "MakeNamedMaterial") {
                std::string n = Str(); ParamSet p = Params();
                std::string type = p.FindOneString("type", "");
                if (type == "") type = gs.materialParams.FindOneString("type", "");
                if (type != "") gs.namedMaterials[n] = MakeMaterial(type, p, gs.materialParams);
            } else if (d == "NamedMaterial") gs.currentNamedMaterial = Str();
            else if (d == "Texture") { std::string n = Str(), type = Str(), cls = Str(); ParamSet p = Params(); MakeTexture(n, type, cls, p); }
            else if (d == "LightSource") { std::string n = Str(); ParamSet p = Params(); MakeLight(n, p); }
            else if (d == "AreaLightSource") { gs.areaLight = Str(); gs.areaLightParams = Params(); }
            else if (d == "Shape") { std::string n = Str(); ParamSet p = Params(); MakeShapeDirective(n, p); }
            else if (d == "Include") {
                std::string fn = Resolve(Str());
                if (havePeek) throw std::runtime_error("internal: include with pending token");
                if (!lex.Include(fn)) throw std::runtime_error("cannot open include " + fn);
            } else if (d == "WorldEnd") { WorldEnd(); worldEnded = true; }
            else if (d == "ObjectBegin" || d == "ObjectInstance" || d == "Volume")
                throw std::runtime_error("unsupported directive in this build: " + d);
            else if (d == "ObjectEnd") {}
            else throw std::runtime_error("unknown directive " + d);
        }
    }

    void LookupCache(const Xform &t, Xform *o2w, Xform *w2o) {   // api.cpp:272-296
        auto it = tcache.find(t);
        if (it == tcache.end()) it = tcache.insert(std::make_pair(t, std::make_pair(t, Xform(Inverse(t))))).first;
        if (o2w) *o2w = it->second.first;
        if (w2o) *w2o = it->second.second;
    }

    // ------------------------------ textures / materials ---------------------------
    int AddTexture(const pbrtgpu_texture &t) {
        out->textures.push_back(t);
        return (int)out->textures.size() - 1;
    }
    static pbrtgpu_texture TexNode(int type, bool spectral) {
        pbrtgpu_texture t{};
        t.type = type; t.spectral = spectral ? 1 : 0;
        t.tex1 = t.tex2 = t.spec = -1;
        t.su = t.sv = 1.f; t.max_aniso = 8.f;
        return t;
    }
    // ReadImage (imageio.cpp:45-66) in this build (no OpenEXR): a .tga / .pfm is decoded (false:
    // the decoder returned NULL), any other file gives the 1x1 RGB 0.5 image
    bool ReadImageFile(const std::string &fn, std::vector<float> &rgb, int *w, int *h) {
        std::string suf = fn.size() >= 5 ? fn.substr(fn.size() - 4) : std::string();
        if (suf == ".tga" || suf == ".TGA") return ReadTGA(fn, rgb, w, h);
        if (suf == ".pfm" || suf == ".PFM") return ReadPFM(fn, rgb, w, h);
        rgb.assign(3, 0.5f);
        *w = *h = 1;
        return true;
    }
    // the 2D mapping of an image or checkerboard texture (imagemap.cpp:107-125, checkerboard.cpp:
    // 36-55): uv (its scales / offsets), spherical and cylindrical (WorldToTexture = Inverse(tex2world),
    // the CTM at the Texture directive), planar (v1, v2 and the udelta / vdelta offsets); an unknown
    // name is the reference's Error + default UVMapping2D
    void ParseMapping(const ParamSet &p, pbrtgpu_texture &t) {
        const std::string mapping = GetString(p, p, "mapping", "uv");
        if (mapping == "uv") {
            t.su = GetFloat(p, p, "uscale", 1.f); t.sv = GetFloat(p, p, "vscale", 1.f);
            t.du = GetFloat(p, p, "udelta", 0.f); t.dv = GetFloat(p, p, "vdelta", 0.f);
        } else if (mapping == "spherical" || mapping == "cylindrical") {
            t.mapping = mapping == "spherical" ? PBRTGPU_MAP_SPHERICAL : PBRTGPU_MAP_CYLINDRICAL;
            const Xform w2t = Inverse(curT.t[0]);
            for (int i = 0; i < 16; ++i) t.map[i] = w2t.m.m[i / 4][i % 4];
        } else if (mapping == "planar") {
            t.mapping = PBRTGPU_MAP_PLANAR;
            const V3 vs = p.FindOneVector("v1", V3(1, 0, 0)), vt = p.FindOneVector("v2", V3(0, 1, 0));
            t.map[0] = vs.x; t.map[1] = vs.y; t.map[2] = vs.z; t.map[3] = vt.x; t.map[4] = vt.y; t.map[5] = vt.z;
            t.du = GetFloat(p, p, "udelta", 0.f); t.dv = GetFloat(p, p, "vdelta", 0.f);
        } else fprintf(stderr, "pbrthost: 2D texture mapping \"%s\" unknown (UVMapping2D)\n", mapping.c_str());
    }
    // ImageTexture (imagemap.cpp:47-73 GetTexture, :97-160 Create*): the image after convertIn --
    // Pow(scale * rgb, gamma) per channel, or powf(scale * rgb.y(), gamma) for a float texture --
    // in a MIPMap pyramid (BuildMipmap) in out->texels; an unreadable .tga / .pfm gives the
    // one-valued MIPMap(1, 1, powf(scale, gamma)) with the MIPMap defaults
    int MakeImageTexture(const ParamSet &p, bool spectral) {
        pbrtgpu_texture t = TexNode(PBRTGPU_TEX_IMAGE, spectral);
        ParseMapping(p, t);
        float maxAniso = GetFloat(p, p, "maxanisotropy", 8.f);
        bool trilerp = p.FindOneBool("trilinear", false), noFilt = p.FindOneBool("noFiltering", false);
        std::string wrap = GetString(p, p, "wrap", "repeat");
        int wm = wrap == "black" ? PBRTGPU_WRAP_BLACK : (wrap == "clamp" ? PBRTGPU_WRAP_CLAMP : PBRTGPU_WRAP_REPEAT);
        float scale = GetFloat(p, p, "scale", 1.f), gamma = GetFloat(p, p, "gamma", 1.f);
        std::string fn = GetString(p, p, "filename", "");
        if (!fn.empty()) fn = Resolve(fn);
        const TexInfoKey key{fn, trilerp, maxAniso, wm, scale, gamma};
        auto hit = mipCache[spectral ? 1 : 0].find(key);
        if (hit != mipCache[spectral ? 1 : 0].end()) {   // the cached MIPMap: its pyramid and flags
            const pbrtgpu_texture &c = hit->second;
            t.texel_off = c.texel_off; t.width = c.width; t.height = c.height; t.levels = c.levels;
            t.trilinear = c.trilinear; t.nofilter = c.nofilter; t.max_aniso = c.max_aniso; t.wrap = c.wrap;
            return AddTexture(t);
        }
        const int nc = spectral ? 3 : 1;
        std::vector<float> rgb, img;
        int w = 0, h = 0;
        t.texel_off = (int)out->texels.size();
        if (ReadImageFile(fn, rgb, &w, &h)) {
            img.resize((size_t)w * h * nc);
            for (size_t i = 0; i < (size_t)w * h; ++i) {
                if (spectral)
                    for (int k = 0; k < 3; ++k) img[3 * i + k] = powf(rgb[3 * i + k] * scale, gamma);
                else   // RGBSpectrum::y(): YWeight . c
                    img[i] = powf(scale * (0.212671f * rgb[3 * i] + 0.715160f * rgb[3 * i + 1] + 0.072169f * rgb[3 * i + 2]),
                                  gamma);
            }
            t.trilinear = (trilerp || noFilt) ? 1 : 0;
            t.nofilter = noFilt ? 1 : 0;
            t.max_aniso = maxAniso;
            t.wrap = wm;
        } else {
            w = h = 1;
            img.assign((size_t)nc, powf(scale, gamma));
            t.trilinear = 0; t.nofilter = 0; t.max_aniso = 8.f; t.wrap = PBRTGPU_WRAP_REPEAT;
        }
        if ((size_t)out->texels.size() + (size_t)w * h * nc * 2 > (size_t)INT32_MAX)
            throw std::runtime_error("image map " + fn + ": texel pool exceeds 2^31 floats");
        BuildMipmap(w, h, std::move(img), nc, t.wrap, out->texels, &t.width, &t.height, &t.levels);
        mipCache[spectral ? 1 : 0][key] = t;
        return AddTexture(t);
    }
    // a Checkerboard2DTexture node: the 2D mapping and the antialiasing mode ("closedform", "none";
    // anything else is the reference's warning + closedform); dimension 3 (Checkerboard3DTexture)
    // is not built
    pbrtgpu_texture CheckerNode(const ParamSet &p, bool spectral) {
        if (p.FindOneInt("dimension", 2) != 2) throw std::runtime_error("3D checkerboard textures are not supported yet");
        pbrtgpu_texture n = TexNode(PBRTGPU_TEX_CHECKER, spectral);
        ParseMapping(p, n);
        const std::string aa = GetString(p, p, "aamode", "closedform");
        if (aa != "none" && aa != "closedform")
            fprintf(stderr, "pbrthost: antialiasing mode \"%s\" not understood by Checkerboard2DTexture; using \"closedform\"\n", aa.c_str());
        n.aamode = aa == "none" ? 1 : 0;
        return n;
    }
    // operands of a checkerboard or mix texture (and a mix's amount): constants become CONST nodes,
    // textures must be image maps (or uv textures)
    int CheckerLeaf(const FloatTex &f) {
        if (f.constant) {
            pbrtgpu_texture t = TexNode(PBRTGPU_TEX_CONST, false);
            t.value = f.value;
            return AddTexture(t);
        }
        if (out->textures[f.tex].type != PBRTGPU_TEX_IMAGE) throw std::runtime_error("checkerboard operands other than constants and image maps are not supported yet");
        return f.tex;
    }
    int CheckerLeaf(const SpecTex &f) {
        if (f.constant) {
            pbrtgpu_texture t = TexNode(PBRTGPU_TEX_CONST, true);
            t.spec = EmitSpectrum(f.value);
            return AddTexture(t);
        }
        if (out->textures[f.tex].type != PBRTGPU_TEX_IMAGE && out->textures[f.tex].type != PBRTGPU_TEX_UV) throw std::runtime_error("checkerboard operands other than constants and image maps are not supported yet");
        return f.tex;
    }
    // operand of a ScaleTexture<float>: a CONST, IMAGE or noise (fbm / wrinkled / windy) node -- the
    // leaf kinds the device evaluates (device.h tex_leaf_float; scene_build.h leafOk)
    int FloatLeaf(const FloatTex &f) {
        if (!f.constant) {
            const int ty = out->textures[f.tex].type;
            if (ty == PBRTGPU_TEX_SCALE) throw std::runtime_error("nested scale textures are not supported yet");
            if (ty != PBRTGPU_TEX_IMAGE && !(ty >= PBRTGPU_TEX_FBM && ty <= PBRTGPU_TEX_WINDY))
                throw std::runtime_error("scale texture operands other than constants, image maps and noise "
                                         "textures are not supported yet");
            return f.tex;
        }
        pbrtgpu_texture t = TexNode(PBRTGPU_TEX_CONST, false);
        t.value = f.value;
        return AddTexture(t);
    }
    void MakeTexture(const std::string &name, const std::string &type, const std::string &cls, const ParamSet &p) {
        // TextureParams(params, params, ...) -- api.cpp:933-956
        if (type == "float") {
            FloatTex t;
            if (cls == "constant") t.value = GetFloat(p, p, "value", 1.f);
            else if (cls == "scale") {   // ScaleTexture::Evaluate = tex1 * tex2 (scale.h)
                FloatTex a = GetFloatTex(p, p, "tex1", 1.f), b = GetFloatTex(p, p, "tex2", 1.f);
                if (a.constant && b.constant) t.value = a.value * b.value;
                else {
                    pbrtgpu_texture n = TexNode(PBRTGPU_TEX_SCALE, false);
                    n.tex1 = FloatLeaf(a); n.tex2 = FloatLeaf(b);
                    t.constant = false; t.tex = AddTexture(n);
                }
            } else if (cls == "imagemap") { t.constant = false; t.tex = MakeImageTexture(p, false); }
            else if (cls == "fbm" || cls == "wrinkled" || cls == "windy") {
                // FBmTexture / WrinkledTexture / WindyTexture<float> (fbm.cpp, wrinkled.cpp, windy.cpp):
                // IdentityMapping3D(tex2world), octaves (8) and roughness (.5)
                pbrtgpu_texture n = TexNode(cls == "fbm" ? PBRTGPU_TEX_FBM : cls == "wrinkled" ? PBRTGPU_TEX_WRINKLED
                                                                                                : PBRTGPU_TEX_WINDY, false);
                for (int i = 0; i < 16; ++i) n.map[i] = curT.t[0].m.m[i / 4][i % 4];
                n.levels = p.FindOneInt("octaves", 8);
                n.value = GetFloat(p, p, "roughness", .5f);
                if (n.levels < 0 || n.levels > 64) throw std::runtime_error("noise texture octaves out of range");
                t.constant = false; t.tex = AddTexture(n);
            }
            else if (cls == "dots") {   // DotsTexture<float> (dots.cpp:30-55): tex1 = "inside", tex2 = "outside"
                pbrtgpu_texture n = TexNode(PBRTGPU_TEX_DOTS, false);
                ParseMapping(p, n);
                n.tex1 = CheckerLeaf(GetFloatTex(p, p, "inside", 1.f));
                n.tex2 = CheckerLeaf(GetFloatTex(p, p, "outside", 0.f));
                t.constant = false; t.tex = AddTexture(n);
            }
            else if (cls == "bilerp") {   // BilerpTexture<float> (bilerp.cpp:30-55): v00 .. v11 in texels[]
                pbrtgpu_texture n = TexNode(PBRTGPU_TEX_BILERP, false);
                ParseMapping(p, n);
                n.texel_off = (int)out->texels.size();
                for (const char *k : {"v00", "v01", "v10", "v11"})
                    out->texels.push_back(GetFloat(p, p, k, (k[2] == '1') ? 1.f : 0.f));
                t.constant = false; t.tex = AddTexture(n);
            }
            else if (cls == "mix") {   // MixTexture<float> (mix.cpp:30-36)
                pbrtgpu_texture n = TexNode(PBRTGPU_TEX_MIX, false);
                n.tex1 = CheckerLeaf(GetFloatTex(p, p, "tex1", 0.f));
                n.tex2 = CheckerLeaf(GetFloatTex(p, p, "tex2", 1.f));
                n.amount = CheckerLeaf(GetFloatTex(p, p, "amount", .5f));
                t.constant = false; t.tex = AddTexture(n);
            }
            else if (cls == "checkerboard") {   // Checkerboard2DTexture<float> (checkerboard.cpp:29-67)
                pbrtgpu_texture n = CheckerNode(p, false);
                n.tex1 = CheckerLeaf(GetFloatTex(p, p, "tex1", 1.f));
                n.tex2 = CheckerLeaf(GetFloatTex(p, p, "tex2", 0.f));
                t.constant = false; t.tex = AddTexture(n);
            }
            else throw std::runtime_error("float texture '" + cls + "' is not supported yet");
            gs.floatTextures[name] = t;
        } else if (type == "color" || type == "spectrum") {
            SpecTex t;
            if (cls == "constant") t.value = GetSpec(p, p, "value", spec.Const(1.f));
            else if (cls == "scale") {
                SpecTex a = GetSpecTex(p, p, "tex1", spec.Const(1.f)), b = GetSpecTex(p, p, "tex2", spec.Const(1.f));
                if (a.constant && b.constant) t.value = SpecMul(a.value, b.value);
                else {
                    // device form: one image leaf times one constant spectrum
                    if (!a.constant && !b.constant) throw std::runtime_error("scale of two non-constant spectrum textures is not supported yet");
                    const SpecTex &img = a.constant ? b : a, &cst = a.constant ? a : b;
                    if (out->textures[img.tex].type != PBRTGPU_TEX_IMAGE && out->textures[img.tex].type != PBRTGPU_TEX_UV)
                        throw std::runtime_error("nested scale textures are not supported yet");
                    pbrtgpu_texture c = TexNode(PBRTGPU_TEX_CONST, true);
                    c.spec = EmitSpectrum(cst.value);
                    int ci = AddTexture(c);
                    pbrtgpu_texture n = TexNode(PBRTGPU_TEX_SCALE, true);
                    n.tex1 = a.constant ? ci : img.tex; n.tex2 = a.constant ? img.tex : ci;
                    t.constant = false; t.tex = AddTexture(n);
                }
            } else if (cls == "imagemap") { t.constant = false; t.tex = MakeImageTexture(p, true); }
            else if (cls == "uv") {   // UVTexture (uv.cpp:37-62): its 2D mapping alone
                pbrtgpu_texture n = TexNode(PBRTGPU_TEX_UV, true);
                ParseMapping(p, n);
                t.constant = false; t.tex = AddTexture(n);
            }
            else if (cls == "fbm" || cls == "wrinkled" || cls == "windy") {   // Texture<Spectrum>: Spectrum(value)
                pbrtgpu_texture n = TexNode(cls == "fbm" ? PBRTGPU_TEX_FBM : cls == "wrinkled" ? PBRTGPU_TEX_WRINKLED
                                                                                                : PBRTGPU_TEX_WINDY, true);
                for (int i = 0; i < 16; ++i) n.map[i] = curT.t[0].m.m[i / 4][i % 4];
                n.levels = p.FindOneInt("octaves", 8);
                n.value = GetFloat(p, p, "roughness", .5f);
                if (n.levels < 0 || n.levels > 64) throw std::runtime_error("noise texture octaves out of range");
                t.constant = false; t.tex = AddTexture(n);
            }
            else if (cls == "marble") {   // MarbleTexture (marble.cpp:37-46), its spline colours FromRGB'd here
                static const float c[9][3] = {{.58f, .58f, .6f}, {.58f, .58f, .6f}, {.58f, .58f, .6f}, {.5f, .5f, .5f},
                                              {.6f, .59f, .58f}, {.58f, .58f, .6f}, {.58f, .58f, .6f}, {.2f, .2f, .33f},
                                              {.58f, .58f, .6f}};   // marble.h:51-53
                pbrtgpu_texture n = TexNode(PBRTGPU_TEX_MARBLE, true);
                for (int i = 0; i < 16; ++i) n.map[i] = curT.t[0].m.m[i / 4][i % 4];
                n.levels = p.FindOneInt("octaves", 8);
                n.value = GetFloat(p, p, "roughness", .5f);
                n.su = GetFloat(p, p, "scale", 1.f);
                n.sv = GetFloat(p, p, "variation", .2f);
                if (n.levels < 0 || n.levels > 64) throw std::runtime_error("marble texture octaves out of range");
                n.spec = -1;
                for (int i = 0; i < 9; ++i) {
                    const int o = EmitSpectrum(spec.FromRGB(c[i]));
                    if (n.spec < 0) n.spec = o;
                }
                t.constant = false; t.tex = AddTexture(n);
            }
            else if (cls == "dots") {   // DotsTexture<Spectrum> (dots.cpp:59-84)
                pbrtgpu_texture n = TexNode(PBRTGPU_TEX_DOTS, true);
                ParseMapping(p, n);
                n.tex1 = CheckerLeaf(GetSpecTex(p, p, "inside", spec.Const(1.f)));
                n.tex2 = CheckerLeaf(GetSpecTex(p, p, "outside", spec.Const(0.f)));
                t.constant = false; t.tex = AddTexture(n);
            }
            else if (cls == "bilerp") {   // BilerpTexture<Spectrum> (bilerp.cpp:59-84): four consecutive spectra
                pbrtgpu_texture n = TexNode(PBRTGPU_TEX_BILERP, true);
                ParseMapping(p, n);
                n.spec = -1;
                for (const char *k : {"v00", "v01", "v10", "v11"}) {
                    const int o = EmitSpectrum(GetSpec(p, p, k, spec.Const((k[2] == '1') ? 1.f : 0.f)));
                    if (n.spec < 0) n.spec = o;
                }
                t.constant = false; t.tex = AddTexture(n);
            }
            else if (cls == "mix") {   // MixTexture<Spectrum> (mix.cpp:40-46)
                pbrtgpu_texture n = TexNode(PBRTGPU_TEX_MIX, true);
                n.tex1 = CheckerLeaf(GetSpecTex(p, p, "tex1", spec.Const(0.f)));
                n.tex2 = CheckerLeaf(GetSpecTex(p, p, "tex2", spec.Const(1.f)));
                n.amount = CheckerLeaf(GetFloatTex(p, p, "amount", .5f));
                t.constant = false; t.tex = AddTexture(n);
            }
            else if (cls == "checkerboard") {   // Checkerboard2DTexture<Spectrum> (checkerboard.cpp:71-110)
                pbrtgpu_texture n = CheckerNode(p, true);
                n.tex1 = CheckerLeaf(GetSpecTex(p, p, "tex1", spec.Const(1.f)));
                n.tex2 = CheckerLeaf(GetSpecTex(p, p, "tex2", spec.Const(0.f)));
                t.constant = false; t.tex = AddTexture(n);
            }
            else throw std::runtime_error("spectrum texture '" + cls + "' is not supported yet");
            gs.spectrumTextures[name] = t;
        }
    }
    float GetFloat(const ParamSet &g, const ParamSet &m, const std::string &n, float d) {
        return g.FindOneFloat(n, m.FindOneFloat(n, d));
    }
    std::string GetString(const ParamSet &g, const ParamSet &m, const std::string &n, const std::string &d) {
        return g.FindOneString(n, m.FindOneString(n, d));   // TextureParams::FindFilename / FindString
    }
    Spec GetSpec(const ParamSet &g, const ParamSet &m, const std::string &n, const Spec &d) {
        return g.FindOneSpectrum(n, m.FindOneSpectrum(n, d));
    }
    FloatTex GetFloatTex(const ParamSet &g, const ParamSet &m, const std::string &n, float d) {   // paramset.cpp:608-622
        std::string name = g.FindTexture(n);
        if (name == "") name = m.FindTexture(n);
        if (name != "") {
            auto it = gs.floatTextures.find(name);
            if (it != gs.floatTextures.end()) return it->second;
            out->warnings.push_back("couldn't find float texture " + name);
        }
        FloatTex t; t.value = GetFloat(g, m, n, d); return t;
    }
    SpecTex GetSpecTex(const ParamSet &g, const ParamSet &m, const std::string &n, const Spec &d) {   // paramset.cpp:591-605
        std::string name = g.FindTexture(n);
        if (name == "") name = m.FindTexture(n);
        if (name != "") {
            auto it = gs.spectrumTextures.find(name);
            if (it != gs.spectrumTextures.end()) return it->second;
            out->warnings.push_back("couldn't find spectrum texture " + name);
        }
        SpecTex t; t.value = GetSpec(g, m, n, d); return t;
    }
    // spectrum parameter k of a material: a constant (clamped where the material clamps) or a
    // textured slot evaluated per hit on the device (`.Clamp()`ed there unless clamp is false:
    // black_mask bit 4 + k); a material has at most two spectrum parameters
    void SpecSlot(MaterialObj &mo, int k, const ParamSet &g, const ParamSet &m, const std::string &n, const Spec &d,
                  bool clamp) {
        SpecTex t = GetSpecTex(g, m, n, d);
        if ((int)mo.spectra.size() != k || k > 1) throw std::runtime_error("internal: material slot order");
        if (t.constant) { mo.spectra.push_back(clamp ? SpecClamp(t.value) : t.value); return; }
        mo.m.tex[k] = t.tex;
        if (!clamp) mo.m.black_mask |= 1 << (4 + k);
        mo.spectra.push_back(spec.Const(0.f));   // placeholder; the device evaluates tex[k]
    }
    // float parameter j (f[0], f[1]) of a material: a constant, or a float texture evaluated per hit
    // on the device (ftex[j]); matte's sigma is clamped to [0, 90] on either side (matte.cpp:54)
    void FloatSlot(MaterialObj &mo, int j, const ParamSet &g, const ParamSet &m, const std::string &n, float d,
                   bool clampSigma = false) {
        FloatTex t = GetFloatTex(g, m, n, d);
        if (t.constant) { mo.m.f[j] = clampSigma ? Clamp(t.value, 0.f, 90.f) : t.value; return; }
        mo.m.ftex[j] = t.tex;
        mo.m.f[j] = 0.f;   // unused: the device evaluates ftex[j]
    }
    std::shared_ptr<MaterialObj> MakeMaterial(const std::string &name, const ParamSet &g, const ParamSet &m) {
        auto mo = std::make_shared<MaterialObj>();
        pbrtgpu_material &mt = mo->m;
        for (int k = 0; k < 4; ++k) mt.tex[k] = -1;
        mt.ftex[0] = mt.ftex[1] = -1;
        mt.bump_tex = -1;
        mt.normal_tex = -1;
        // every material: normalmap (Material::NormalMap where its value is not black; the default
        // constant 0 never is) and bumpmap (float texture)
        SpecTex nmap = GetSpecTex(g, m, "normalmap", spec.Const(0.f));
        if (nmap.constant) {
            if (!SpecIsBlack(nmap.value)) {   // EvaluateMemory of a constant is RGB 0 (constant.h:45-47)
                pbrtgpu_texture c = TexNode(PBRTGPU_TEX_CONST, true);
                c.spec = EmitSpectrum(nmap.value);
                mt.normal_tex = AddTexture(c);
            }
        } else mt.normal_tex = nmap.tex;
        FloatTex bump = GetFloatTex(g, m, "bumpmap", 0.f);
        if (bump.constant) mt.f[7] = bump.value;
        else mt.bump_tex = bump.tex;
        if (name == "matte") {   // matte.cpp:34-72
            mt.type = PBRTGPU_MAT_MATTE;
            SpecSlot(*mo, 0, g, m, "Kd", spec.Const(0.5f), true);
            FloatSlot(*mo, 0, g, m, "sigma", 0.f, true);
        } else if (name == "plastic") {   // plastic.cpp:34-74
            mt.type = PBRTGPU_MAT_PLASTIC;
            SpecSlot(*mo, 0, g, m, "Kd", spec.Const(0.25f), true);
            SpecSlot(*mo, 1, g, m, "Ks", spec.Const(0.25f), true);
            FloatSlot(*mo, 0, g, m, "roughness", .1f);
        } else if (name == "mirror") {   // mirror.cpp
            mt.type = PBRTGPU_MAT_MIRROR;
            SpecSlot(*mo, 0, g, m, "Kr", spec.Const(0.9f), true);
        } else if (name == "shinymetal") {   // shinymetal.cpp:31-38 FresnelApproxEta, 45-84
            mt.type = PBRTGPU_MAT_SHINYMETAL;
            SpecTex kr = GetSpecTex(g, m, "Kr", spec.Const(1.f)), ks = GetSpecTex(g, m, "Ks", spec.Const(1.f));
            if (!kr.constant || !ks.constant) throw std::runtime_error("shinymetal: textured Kr / Ks are not supported yet");
            auto approxEta = [](const Spec &fr) {   // (1 + Sqrt(r)) / (1 - Sqrt(r)), r = Fr.Clamp(0, .999)
                Spec e(fr.size());
                for (size_t i = 0; i < fr.size(); ++i) {
                    const float r = Clamp(fr[i], 0.f, .999f);
                    e[i] = (1.f + sqrtf(r)) / (1.f - sqrtf(r));
                }
                return e;
            };
            mo->spectra.push_back(approxEta(SpecClamp(ks.value)));   // Ks->Evaluate(dgs).Clamp()
            mo->spectra.push_back(approxEta(SpecClamp(kr.value)));   // Kr->Evaluate(dgs).Clamp()
            mo->spectra.push_back(spec.Const(0.f));                  // k = 0.
            FloatSlot(*mo, 0, g, m, "roughness", .1f);
        } else if (name == "anisoward") {   // anisoward.cpp:62-74 (the fork's anisotropic Ward material)
            mt.type = PBRTGPU_MAT_ANISOWARD;
            SpecSlot(*mo, 0, g, m, "Kd", spec.Const(0.25f), true);
            SpecSlot(*mo, 1, g, m, "Ks", spec.Const(0.25f), true);
            FloatSlot(*mo, 0, g, m, "alphaU", .1f);
            FloatSlot(*mo, 1, g, m, "alphaV", .1f);
        } else if (name == "substrate") {   // substrate.cpp
            mt.type = PBRTGPU_MAT_SUBSTRATE;
            SpecSlot(*mo, 0, g, m, "Kd", spec.Const(.5f), true);
            SpecSlot(*mo, 1, g, m, "Ks", spec.Const(.5f), true);
            FloatSlot(*mo, 0, g, m, "uroughness", .1f);
            FloatSlot(*mo, 1, g, m, "vroughness", .1f);
        } else if (name == "glass") {   // glass.cpp:34-68
            mt.type = PBRTGPU_MAT_GLASS;
            SpecSlot(*mo, 0, g, m, "Kr", spec.Const(1.f), true);
            SpecSlot(*mo, 1, g, m, "Kt", spec.Const(1.f), true);
            FloatSlot(*mo, 0, g, m, "index", 1.5f);
        } else if (name == "metal") {   // metal.cpp:44-62, 99-110 (eta, k unclamped)
            mt.type = PBRTGPU_MAT_METAL;
            SpecSlot(*mo, 0, g, m, "eta", CopperSpectrum(false), false);
            SpecSlot(*mo, 1, g, m, "k", CopperSpectrum(true), false);
            FloatSlot(*mo, 0, g, m, "roughness", .01f);
        } else if (name == "measured") {   // measured.cpp:66-130, 182-206 (.brdf: IrregIsotropicBRDF)
            mt.type = PBRTGPU_MAT_MEASURED;
            std::string fn = Resolve(GetString(g, m, "filename", ""));
            size_t dot = fn.rfind('.');
            std::string suf = dot == std::string::npos ? "" : fn.substr(dot);
            if (suf == ".brdf" || suf == ".BRDF") {
                auto it = measuredCache.find(fn);
                if (it == measuredCache.end()) it = measuredCache.insert(std::make_pair(fn, LoadIrregBrdf(fn))).first;
                mo->measured = it->second;
            } else {
                // any other suffix: the MERL RegularHalfangle format (measured.cpp:131-175)
                mt.type = PBRTGPU_MAT_MEASURED_HALFANGLE;
                auto it = merlCache.find(fn);
                if (it == merlCache.end()) it = merlCache.insert(std::make_pair(fn, LoadMerl(fn))).first;
                mt.aux = it->second;
            }
        } else
            throw std::runtime_error("material '" + name + "' is not supported by this build yet");
        mo->refId = nextMatId++;
        return mo;
    }
    // default metal eta / k: copper, sampled at 56 wavelengths (metal.cpp:71-97), FromSampled
    Spec CopperSpectrum(bool kAbsorption) const {
        static const float wl[56] = {
        298.7570554f, 302.4004341f, 306.1337728f, 309.960445f, 313.8839949f, 317.9081487f, 322.036826f,
        326.2741526f, 330.6244747f, 335.092373f, 339.6826795f, 344.4004944f, 349.2512056f, 354.2405086f,
        359.374429f, 364.6593471f, 370.1020239f, 375.7096303f, 381.4897785f, 387.4505563f, 393.6005651f,
        399.9489613f, 406.5055016f, 413.2805933f, 420.2853492f, 427.5316483f, 435.0322035f, 442.8006357f,
        450.8515564f, 459.2006593f, 467.8648226f, 476.8622231f, 486.2124627f, 495.936712f, 506.0578694f,
        516.6007417f, 527.5922468f, 539.0616435f, 551.0407911f, 563.5644455f, 576.6705953f, 590.4008476f,
        604.8008683f, 619.92089f, 635.8162974f, 652.5483053f, 670.1847459f, 688.8009889f, 708.4810171f,
        729.3186941f, 751.4192606f, 774.9011125f, 799.8979226f, 826.5611867f, 855.0632966f, 885.6012714f};
        static const float eta[56] = {
        1.400313f, 1.38f, 1.358438f, 1.34f, 1.329063f, 1.325f, 1.3325f, 1.34f, 1.334375f, 1.325f, 1.317812f,
        1.31f, 1.300313f, 1.29f, 1.281563f, 1.27f, 1.249062f, 1.225f, 1.2f, 1.18f, 1.174375f, 1.175f,
        1.1775f, 1.18f, 1.178125f, 1.175f, 1.172812f, 1.17f, 1.165312f, 1.16f, 1.155312f, 1.15f, 1.142812f,
        1.135f, 1.131562f, 1.12f, 1.092437f, 1.04f, 0.950375f, 0.826f, 0.645875f, 0.468f, 0.35125f, 0.272f,
        0.230813f, 0.214f, 0.20925f, 0.213f, 0.21625f, 0.223f, 0.2365f, 0.25f, 0.254188f, 0.26f, 0.28f, 0.3f};
        static const float kk[56] = {
        1.662125f, 1.687f, 1.703313f, 1.72f, 1.744563f, 1.77f, 1.791625f, 1.81f, 1.822125f, 1.834f, 1.85175f,
        1.872f, 1.89425f, 1.916f, 1.931688f, 1.95f, 1.972438f, 2.015f, 2.121562f, 2.21f, 2.177188f, 2.13f,
        2.160063f, 2.21f, 2.249938f, 2.289f, 2.326f, 2.362f, 2.397625f, 2.433f, 2.469187f, 2.504f, 2.535875f,
        2.564f, 2.589625f, 2.605f, 2.595562f, 2.583f, 2.5765f, 2.599f, 2.678062f, 2.809f, 3.01075f, 3.24f,
        3.458187f, 3.67f, 3.863125f, 4.05f, 4.239563f, 4.43f, 4.619563f, 4.817f, 5.034125f, 5.26f, 5.485625f,
        5.717f};
        return spec.FromSampled(wl, kAbsorption ? kk : eta, 56);
    }
    std::map<std::string, std::shared_ptr<MeasuredData> > measuredCache;
    // ImageTexture::GetTexture's MIPMap cache (imagemap.cpp:47-80, imagemap.h:39-55), one per
    // ImageTexture instantiation (float, spectrum): keyed by TexInfo -- filename, doTrilinear,
    // maxAniso, wrap, scale, gamma, NOT noFiltering -- so a later texture with the same key takes
    // the first one's MIPMap, its pyramid and its filtering flags; the value is that texture record
    struct TexInfoKey {
        std::string filename;
        bool trilinear;
        float maxAniso;
        int wrap;
        float scale, gamma;
        bool operator<(const TexInfoKey &o) const {   // TexInfo::operator< (its field order)
            if (filename != o.filename) return filename < o.filename;
            if (trilinear != o.trilinear) return trilinear < o.trilinear;
            if (maxAniso != o.maxAniso) return maxAniso < o.maxAniso;
            if (scale != o.scale) return scale < o.scale;
            if (gamma != o.gamma) return gamma < o.gamma;
            return wrap < o.wrap;
        }
    };
    std::map<TexInfoKey, pbrtgpu_texture> mipCache[2];
    std::map<std::string, int> merlCache;   // loadedRegularHalfangle (measured.cpp:99)
    // ReadFloatFile (floatfile.cpp:30-74)
    static std::vector<float> ReadFloatFile(const std::string &fn) {
        FILE *fp = fopen(fn.c_str(), "r");
        if (!fp) throw std::runtime_error("Unable to open file " + fn);
        std::vector<float> values;
        int c;
        bool inNumber = false;
        char cur[32];
        int pos = 0;
        while ((c = getc(fp)) != EOF) {
            if (inNumber) {
                if (isdigit(c) || c == '.' || c == 'e' || c == '-' || c == '+') { if (pos < 31) cur[pos++] = (char)c; }
                else { cur[pos] = 0; values.push_back((float)atof(cur)); inNumber = false; pos = 0; }
            } else {
                if (isdigit(c) || c == '.' || c == '-' || c == '+') { inNumber = true; cur[pos++] = (char)c; }
                else if (c == '#') { while ((c = getc(fp)) != '\n' && c != EOF) {} }
            }
        }
        fclose(fp);
        return values;
    }
    // BRDFRemap (reflection.cpp:239-248); pbrt.h:179 defines M_PI as a float literal, so
    // everything is single precision
    static V3 BRDFRemap(const V3 &wo, const V3 &wi) {
        const float kPiF = 3.14159265358979323846f;
        float cosi = wi.z, coso = wo.z;
        float sini = sqrtf(pmax(0.f, 1.f - cosi * cosi)), sino = sqrtf(pmax(0.f, 1.f - coso * coso));
        float pi_ = atan2f(wi.y, wi.x); float phii = (pi_ < 0.f) ? pi_ + 2.f * kPiF : pi_;
        float po_ = atan2f(wo.y, wo.x); float phio = (po_ < 0.f) ? po_ + 2.f * kPiF : po_;
        float dphi = phii - phio;
        if (dphi < 0.) dphi += 2.f * kPiF;
        if (dphi > 2.f * kPiF) dphi -= 2.f * kPiF;
        if (dphi > kPiF) dphi = 2.f * kPiF - dphi;
        return V3(sini * sino, dphi / kPiF, cosi * coso);
    }
    // RegularHalfangle data (measured.cpp:131-175): three int dims whose product must be
    // 90 * 90 * 180, then per RGB channel that many doubles in chunks of 2 * nPhiD, each
    // scaled (1/1500, 1.15/1500, 1.66/1500 as float constants) and clamped at 0 in double,
    // stored as float.  Returns the first texel in out->merl, or -1 when the reference's loader
    // fails (Error(); the material then has no BxDF).
    int LoadMerl(const std::string &fn) {
        const uint32_t nThetaH = 90, nThetaD = 90, nPhiD = 180;
        FILE *f = fopen(fn.c_str(), "rb");
        if (!f) { out->warnings.push_back("Unable to open BRDF data file " + fn); return -1; }
        int dims[3];
        if (fread(dims, sizeof(int), 3, f) != 3) {
            out->warnings.push_back("Premature end-of-file in measured BRDF data file " + fn);
            fclose(f);
            return -1;
        }
        const uint32_t n = (uint32_t)dims[0] * (uint32_t)dims[1] * (uint32_t)dims[2];
        if (n != nThetaH * nThetaD * nPhiD) {
            out->warnings.push_back("Dimensions don't match in " + fn);
            fclose(f);
            return -1;
        }
        std::vector<float> tab(3 * (size_t)n);
        const uint32_t chunkSize = 2 * nPhiD, nChunks = n / chunkSize;
        std::vector<double> tmp(chunkSize);
        const float scales[3] = {1.f / 1500.f, 1.15f / 1500.f, 1.66f / 1500.f};
        for (int c = 0; c < 3; ++c) {
            size_t offset = 0;
            for (uint32_t i = 0; i < nChunks; ++i) {
                if (fread(tmp.data(), sizeof(double), chunkSize, f) != chunkSize) {
                    out->warnings.push_back("Premature end-of-file in measured BRDF data file " + fn);
                    fclose(f);
                    return -1;
                }
                for (uint32_t j = 0; j < chunkSize; ++j) tab[3 * offset++ + c] = (float)std::max(0., tmp[j] * scales[c]);
            }
        }
        fclose(f);
        const int first = (int)(out->merl.size() / 3);
        out->merl.insert(out->merl.end(), tab.begin(), tab.end());
        return first;
    }
    std::shared_ptr<MeasuredData> LoadIrregBrdf(const std::string &fn) {
        std::vector<float> values = ReadFloatFile(fn);
        if (values.empty()) throw std::runtime_error("Unable to read BRDF data from file " + fn);
        size_t pos = 0;
        int numWls = (int)values[pos++];
        if ((values.size() - 1 - numWls) % (4 + numWls) != 0)
            throw std::runtime_error("Excess or insufficient data in theta, phi BRDF file " + fn);
        std::vector<float> wls(values.begin() + 1, values.begin() + 1 + numWls);
        pos += numWls;
        auto md = std::make_shared<MeasuredData>();
        while (pos < values.size()) {
            float thetai = values[pos++], phii = values[pos++], thetao = values[pos++], phio = values[pos++];
            V3 wo(sinf(thetao) * cosf(phio), sinf(thetao) * sinf(phio), cosf(thetao));   // SphericalDirection
            V3 wi(sinf(thetai) * cosf(phii), sinf(thetai) * sinf(phii), cosf(thetai));
            BrdfSample s;
            s.v = spec.FromSampled(wls.data(), &values[pos], numWls);
            pos += numWls;
            s.p = BRDFRemap(wo, wi);
            md->samples.push_back(s);
        }
        return md;
    }
    // KdTree construction (kdtree.h:100-148) into out->kdnodes
    void KdBuild(std::vector<pbrtgpu_kdnode> &nodes, std::vector<int> &nodeSample, uint32_t nodeNum, int start, int end,
                 const BrdfSample **bn, uint32_t *nextFree, const BrdfSample *base) {
        if (start + 1 == end) {
            nodes[nodeNum].split_axis = 3; nodes[nodeNum].right_child = (1 << 29) - 1; nodes[nodeNum].has_left = 0;
            nodeSample[nodeNum] = (int)(bn[start] - base);
            return;
        }
        BBox bound;
        for (int i = start; i < end; ++i) bound = Union(bound, bn[i]->p);
        int axis = bound.MaximumExtent();
        int splitPos = (start + end) / 2;
        std::nth_element(&bn[start], &bn[splitPos], &bn[end], [axis](const BrdfSample *a, const BrdfSample *b) {
            return a->p[axis] == b->p[axis] ? (a < b) : a->p[axis] < b->p[axis];
        });
        nodes[nodeNum].split_pos = bn[splitPos]->p[axis];
        nodes[nodeNum].split_axis = axis;
        nodes[nodeNum].right_child = (1 << 29) - 1;
        nodes[nodeNum].has_left = 0;
        nodeSample[nodeNum] = (int)(bn[splitPos] - base);
        if (start < splitPos) {
            nodes[nodeNum].has_left = 1;
            uint32_t child = (*nextFree)++;
            KdBuild(nodes, nodeSample, child, start, splitPos, bn, nextFree, base);
        }
        if (splitPos + 1 < end) {
            nodes[nodeNum].right_child = (int)(*nextFree)++;
            KdBuild(nodes, nodeSample, nodes[nodeNum].right_child, splitPos + 1, end, bn, nextFree, base);
        }
    }
    int EmitMeasured(MeasuredData *md, int *count) {
        int n = (int)md->samples.size();
        *count = n;
        if (md->flatFirst >= 0) return md->flatFirst;
        std::vector<pbrtgpu_kdnode> nodes(n);
        std::vector<int> nodeSample(n, -1);
        std::vector<const BrdfSample *> bn(n);
        for (int i = 0; i < n; ++i) bn[i] = &md->samples[i];
        uint32_t nextFree = 1;
        if (n > 0) KdBuild(nodes, nodeSample, 0, 0, n, bn.data(), &nextFree, md->samples.data());
        for (int i = 0; i < n; ++i) {
            const BrdfSample &s = md->samples[nodeSample[i]];
            for (int k = 0; k < 3; ++k) nodes[i].p[k] = s.p[k];
            nodes[i].spec = EmitSpectrum(s.v);
        }
        md->flatFirst = (int)out->kdnodes.size();
        out->kdnodes.insert(out->kdnodes.end(), nodes.begin(), nodes.end());
        return md->flatFirst;
    }
    std::shared_ptr<MaterialObj> CreateMaterialFromState(const ParamSet &params) {   // api.cpp:1127-1143
        if (gs.currentNamedMaterial != "") {
            auto it = gs.namedMaterials.find(gs.currentNamedMaterial);
            if (it != gs.namedMaterials.end() && it->second) return it->second;
        }
        return MakeMaterial(gs.material, params, gs.materialParams);
    }

    // ------------------------------ lights ------------------------------------------
    void MakeLight(const std::string &name, const ParamSet &p) {
        auto lo = std::make_shared<LightObj>();
        if (name == "point") {   // point.cpp:34-40, 69-76
            Spec I = p.FindOneSpectrum("I", spec.Const(1.0f));
            Spec sc = p.FindOneSpectrum("scale", spec.Const(1.0f));
            V3 P = p.FindOnePoint("from", V3(0, 0, 0));
            Xform l2w = Translate(V3(P.x, P.y, P.z)) * curT.t[0];
            lo->l.type = PBRTGPU_LIGHT_POINT;
            lo->L = SpecMul(I, sc);
            V3 lp = l2w.Point(V3(0, 0, 0));
            lo->l.pos[0] = lp.x; lo->l.pos[1] = lp.y; lo->l.pos[2] = lp.z;
            memcpy(lo->l.l2w_m, l2w.m.m, 64); memcpy(lo->l.l2w_minv, l2w.mInv.m, 64);
        } else if (name == "spot") {   // spot.cpp:32-38, 70-92
            Spec I = p.FindOneSpectrum("I", spec.Const(1.0f));
            Spec sc = p.FindOneSpectrum("scale", spec.Const(1.0f));
            const float coneangle = p.FindOneFloat("coneangle", 30.f);
            const float conedelta = p.FindOneFloat("conedeltaangle", 5.f);
            const V3 from = p.FindOnePoint("from", V3(0, 0, 0)), to = p.FindOnePoint("to", V3(0, 0, 1));
            const V3 dir = Normalize(to - from);
            V3 du, dv;
            CoordinateSystem(dir, &du, &dv);
            M4 d2z;
            const float rows[4][4] = {{du.x, du.y, du.z, 0.f}, {dv.x, dv.y, dv.z, 0.f}, {dir.x, dir.y, dir.z, 0.f}, {0.f, 0.f, 0.f, 1.f}};
            for (int i = 0; i < 4; ++i)
                for (int j = 0; j < 4; ++j) d2z.m[i][j] = rows[i][j];
            const Xform dirToZ(d2z);
            const Xform l2w = curT.t[0] * Translate(V3(from.x, from.y, from.z)) * Inverse(dirToZ);
            lo->l.type = PBRTGPU_LIGHT_SPOT;
            lo->L = SpecMul(I, sc);
            const V3 lp = l2w.Point(V3(0, 0, 0));
            lo->l.pos[0] = lp.x; lo->l.pos[1] = lp.y; lo->l.pos[2] = lp.z;
            lo->l.texel[0] = cosf(Radians(coneangle));               // cosTotalWidth
            lo->l.texel[1] = cosf(Radians(coneangle - conedelta));   // cosFalloffStart
            memcpy(lo->l.l2w_m, l2w.m.m, 64); memcpy(lo->l.l2w_minv, l2w.mInv.m, 64);
        } else if (name == "distant") {   // distant.cpp:31-36, 56-64
            Spec L = p.FindOneSpectrum("L", spec.Const(1.0f));
            Spec sc = p.FindOneSpectrum("scale", spec.Const(1.0f));
            const V3 from = p.FindOnePoint("from", V3(0, 0, 0)), to = p.FindOnePoint("to", V3(0, 0, 1));
            const Xform &l2w = curT.t[0];
            lo->l.type = PBRTGPU_LIGHT_DISTANT;
            lo->L = SpecMul(L, sc);
            const V3 d = Normalize(l2w.Vector(from - to));   // lightDir
            lo->l.pos[0] = d.x; lo->l.pos[1] = d.y; lo->l.pos[2] = d.z;
            memcpy(lo->l.l2w_m, l2w.m.m, 64); memcpy(lo->l.l2w_minv, l2w.mInv.m, 64);
        } else if (name == "infinite" || name == "exinfinite") {   // infinite.cpp:41-80, 232-245
            Spec L = p.FindOneSpectrum("L", spec.Const(1.0f));
            Spec sc = p.FindOneSpectrum("scale", spec.Const(1.0f));
            std::string texmap = p.FindOneString("mapname", "");
            lo->l.type = PBRTGPU_LIGHT_INFINITE;
            lo->L = SpecMul(L, sc);
            float rgb[3];
            spec.ToRGB(lo->L, rgb);   // L.ToRGBSpectrum()
            float texel[3] = {rgb[0], rgb[1], rgb[2]};
            lo->l.map_tex = -1;
            lo->l.dist_off = -1;
            lo->l.dist_nu = lo->l.dist_nv = 1;
            lo->l.wrap = PBRTGPU_WRAP_REPEAT;
            if (texmap != "") {   // ReadImage (imageio.cpp:45-66): NULL keeps the one texel L
                std::vector<float> img;
                int w = 0, h = 0;
                if (ReadImageFile(Resolve(texmap), img, &w, &h)) {
                    for (size_t i = 0; i < (size_t)w * h; ++i)   // texels[i] *= L.ToRGBSpectrum()
                        for (int k = 0; k < 3; ++k) img[3 * i + k] *= rgb[k];
                    if (w == 1 && h == 1) for (int k = 0; k < 3; ++k) texel[k] = img[k];
                    else EnvMap(lo->l, w, h, std::move(img));
                }
            }
            for (int k = 0; k < 3; ++k) lo->l.texel[k] = texel[k];
            // Distribution2D of img[0] = Lookup(0, 0, 1).y() * sinTheta (one texel: Texel(0, 0, 0));
            // unused with a decoded map (EnvMap's distribution)
            const float kPiF = 3.14159265358979323846f;
            float img = 0.212671f * texel[0] + 0.715160f * texel[1] + 0.072169f * texel[2];
            img *= sinf(kPiF * float(0 + .5f) / float(1));
            float funcInt = 0.f + img / 1;             // Distribution1D: cdf[1]
            float margFunc = funcInt, margInt = 0.f + margFunc / 1;
            lo->l.map_pdf = (img / funcInt) * (margFunc / margInt);   // SampleContinuous pdfs[0] * pdfs[1]
            lo->l.dist_pdf = (funcInt * margInt == 0.f) ? 0.f : (img * margFunc) / (funcInt * margInt);
            const Xform &l2w = curT.t[0];
            memcpy(lo->l.l2w_m, l2w.m.m, 64); memcpy(lo->l.l2w_minv, l2w.mInv.m, 64);
        } else
            throw std::runtime_error("light '" + name + "' is not supported by this build yet");
        lo->l.is_black = SpecIsBlack(lo->L);
        // Light::nSamples (light.h:45): point lights take none, infinite "nsamples" (infinite.cpp:181)
        lo->l.n_samples = std::max(1, name == "point" ? 1 : p.FindOneInt("nsamples", 1));
        lights.push_back(lo);
    }
    // InfiniteAreaLight's constructor for a decoded environment image (infinite.cpp:60-109): the
    // radiance MIPMap<RGBSpectrum>(width, height, texels) with the MIPMap defaults (no trilinear,
    // max anisotropy 8, repeat; BuildMipmap resamples a non-power-of-two image and clamps it), then
    // the scalar image img[u + v w] = radianceMap->Lookup(u / w, v / h, 1 / max(w, h)).y() *
    // sinf(M_PI * (v + .5) / h) and its Distribution2D, stored after the pyramid in the texel pool
    void EnvMap(pbrtgpu_light &l, int w, int h, std::vector<float> img) {
        pbrtgpu_texture t = TexNode(PBRTGPU_TEX_IMAGE, true);
        t.trilinear = 0; t.nofilter = 0; t.max_aniso = 8.f; t.wrap = PBRTGPU_WRAP_REPEAT;
        t.texel_off = (int)out->texels.size();
        if ((size_t)out->texels.size() + (size_t)w * h * 3 * 2 + (size_t)(w + 2) * (h + 2) * 2 > (size_t)INT32_MAX)
            throw std::runtime_error("environment map: texel pool exceeds 2^31 floats");
        BuildMipmap(w, h, std::move(img), 3, t.wrap, out->texels, &t.width, &t.height, &t.levels);
        l.map_tex = AddTexture(t);
        l.dist_nu = w;
        l.dist_nv = h;
        const float kPiF = 3.14159265358979323846f;   // pbrt.h:179: M_PI is a float literal here
        const float filter = 1.f / std::max(w, h);
        std::vector<float> f((size_t)w * h);
        for (int v = 0; v < h; ++v) {
            const float vp = (float)v / (float)h;
            const float sinTheta = sinf(kPiF * float(v + .5f) / float(h));
            for (int u = 0; u < w; ++u) {
                const float up = (float)u / (float)w;
                float c[3];
                MipLookupW(t, up, vp, filter, c);
                f[u + (size_t)v * w] = 0.212671f * c[0] + 0.715160f * c[1] + 0.072169f * c[2];   // RGBSpectrum::y()
                f[u + (size_t)v * w] *= sinTheta;
            }
        }
        // Distribution2D (montecarlo.cpp:350-362): a Distribution1D per row, then the marginal of
        // their integrals; Distribution1D (montecarlo.h:45-66) in the reference's float order
        auto dist1d = [](const float *fn, int n, std::vector<float> &o) {   // {funcInt, func[n], cdf[n + 1]}
            std::vector<float> cdf(n + 1);
            cdf[0] = 0.;
            for (int i = 1; i < n + 1; ++i) cdf[i] = cdf[i - 1] + fn[i - 1] / n;
            const float funcInt = cdf[n];
            if (funcInt == 0.f) for (int i = 1; i < n + 1; ++i) cdf[i] = float(i) / float(n);
            else for (int i = 1; i < n + 1; ++i) cdf[i] /= funcInt;
            o.push_back(funcInt);
            o.insert(o.end(), fn, fn + n);
            o.insert(o.end(), cdf.begin(), cdf.end());
            return funcInt;
        };
        std::vector<float> rows, marg((size_t)h);
        for (int v = 0; v < h; ++v) marg[v] = dist1d(&f[(size_t)v * w], w, rows);
        l.dist_off = (int)out->texels.size();
        dist1d(marg.data(), h, out->texels);
        out->texels.insert(out->texels.end(), rows.begin(), rows.end());
    }
    // MIPMap::Lookup(s, t, width) (mipmap.h:226-259) of an IMAGE texture's pyramid in the texel pool:
    // the level from the width, triangle filters (mipmap.h:263-274) at one or two levels, Texel's
    // wrap (mipmap.h:197-222); as the device's mip_lookup_w
    void MipLookupW(const pbrtgpu_texture &t, float s, float tt, float width, float res[3]) const {
        const int nc = 3;
        auto level = [&](int lv, const float **T, int *w, int *h) {
            size_t off = (size_t)t.texel_off;
            int ww = t.width, hh = t.height;
            for (int i = 0; i < lv; ++i) { off += (size_t)ww * hh * nc; ww = ww > 1 ? ww >> 1 : 1; hh = hh > 1 ? hh >> 1 : 1; }
            *T = out->texels.data() + off; *w = ww; *h = hh;
        };
        auto texel = [&](const float *T, int w, int h, int s0, int t0, float *o) {
            if (t.wrap == PBRTGPU_WRAP_REPEAT) {
                auto mod = [](int a, int b) { int n = int(a / b); a -= n * b; if (a < 0) a += b; return a; };
                s0 = mod(s0, w); t0 = mod(t0, h);
            } else if (t.wrap == PBRTGPU_WRAP_CLAMP) { s0 = std::min(std::max(s0, 0), w - 1); t0 = std::min(std::max(t0, 0), h - 1); }
            else if (s0 < 0 || s0 >= w || t0 < 0 || t0 >= h) { o[0] = o[1] = o[2] = 0.f; return; }
            for (int k = 0; k < nc; ++k) o[k] = T[((size_t)t0 * w + s0) * nc + k];
        };
        auto tri = [&](int lv, float s, float tv, float *o) {
            lv = std::min(std::max(lv, 0), t.levels - 1);
            const float *T; int w, h;
            level(lv, &T, &w, &h);
            s = s * (float)w - 0.5f;
            tv = tv * (float)h - 0.5f;
            const int s0 = Floor2Int(s), t0 = Floor2Int(tv);
            const float ds = s - s0, dt = tv - t0;
            const float w00 = (1.f - ds) * (1.f - dt), w01 = (1.f - ds) * dt, w10 = ds * (1.f - dt), w11 = ds * dt;
            float a[3], b[3], c[3], d[3];
            texel(T, w, h, s0, t0, a); texel(T, w, h, s0, t0 + 1, b); texel(T, w, h, s0 + 1, t0, c); texel(T, w, h, s0 + 1, t0 + 1, d);
            for (int k = 0; k < nc; ++k) o[k] = ((w00 * a[k] + w01 * b[k]) + w10 * c[k]) + w11 * d[k];
        };
        const float invLog2 = 1.f / logf(2.f);
        const float lvl = (float)(t.levels - 1) + logf(std::max(width, 1e-8f)) * invLog2;   // Log2 (pbrt.h:243-246)
        if (lvl < 0) tri(0, s, tt, res);
        else if (lvl >= (float)(t.levels - 1)) {
            const float *T; int w, h;
            level(t.levels - 1, &T, &w, &h);
            texel(T, w, h, 0, 0, res);
        } else {
            const int il = Floor2Int(lvl);
            const float delta = lvl - il;
            float a[3], b[3];
            tri(il, s, tt, a);
            tri(il + 1, s, tt, b);
            for (int k = 0; k < nc; ++k) res[k] = (1.f - delta) * a[k] + delta * b[k];
        }
    }
    // ShapeSet (light.cpp:114-135): refine with a LIFO todo list
    void ShapeSetOf(const std::shared_ptr<ShapeObj> &s, std::vector<Isect> *set) {
        std::vector<Isect> r;
        RefineShape(s, &r);
        for (auto it = r.rbegin(); it != r.rend(); ++it) set->push_back(*it);
    }

    // ------------------------------ shapes ------------------------------------------
    std::shared_ptr<ShapeObj> MakeShape(const std::string &name, const Xform &o2w, const Xform &w2o, bool ro,
                                        const ParamSet &p) {
        (void)w2o;
        auto s = std::make_shared<ShapeObj>();
        if (name == "trianglemesh") {   // trianglemesh.cpp:363-433
            const Param *vi = p.Find(P_INT, "indices"), *P = p.Find(P_POINT, "P");
            const Param *uvs = p.Find(P_FLOAT, "uv");
            if (!uvs) uvs = p.Find(P_FLOAT, "st");
            if (!vi || !P) return nullptr;
            int npi = (int)P->f.size() / 3;
            std::vector<float> uv;
            if (uvs) {
                if ((int)uvs->f.size() < 2 * npi) out->warnings.push_back("not enough uvs; discarding");
                else uv.assign(uvs->f.begin(), uvs->f.begin() + 2 * npi);
            }
            const Param *N = p.Find(P_NORMAL, "N");
            if (N && (int)N->f.size() / 3 != npi) N = nullptr;
            if (p.Find(P_VECTOR, "S")) throw std::runtime_error("trianglemesh 'S' tangents are not supported yet");
            if (p.FindTexture("alpha") != "" || p.FindOneFloat("alpha", 1.f) == 0.f)
                throw std::runtime_error("alpha textures are not supported yet");
            for (int v : vi->i) if (v >= npi) throw std::runtime_error("trianglemesh index out of bounds");
            auto m = std::make_shared<TriMesh>();
            m->o2w = o2w; m->ro = ro; m->swaps = o2w.SwapsHandedness();
            m->ntris = (int)vi->i.size() / 3; m->nverts = npi;
            m->vi.assign(vi->i.begin(), vi->i.begin() + 3 * m->ntris);
            m->p.resize(npi);
            for (int i = 0; i < npi; ++i) m->p[i] = o2w.Point(V3(P->f[3 * i], P->f[3 * i + 1], P->f[3 * i + 2]));
            if (N) { m->n.resize(npi); for (int i = 0; i < npi; ++i) m->n[i] = V3(N->f[3 * i], N->f[3 * i + 1], N->f[3 * i + 2]); }
            m->uv = uv;
            s->kind = ShapeObj::MESH; s->mesh = m;
            allMeshes.push_back(m);
        } else if (name == "heightfield") {   // heightfield.cpp:55-113: Refine -> one TriangleMesh
            const int nu = p.FindOneInt("nu", -1), nv = p.FindOneInt("nv", -1);
            const Param *Pz = p.Find(P_FLOAT, "Pz");
            if (nu < 2 || nv < 2 || !Pz || (int64_t)Pz->f.size() != (int64_t)nu * nv)
                throw std::runtime_error("heightfield: \"nu\" x \"nv\" \"Pz\" values required");
            auto m = std::make_shared<TriMesh>();
            m->o2w = o2w; m->ro = ro; m->swaps = o2w.SwapsHandedness();
            m->nverts = nu * nv;
            m->ntris = 2 * (nu - 1) * (nv - 1);
            m->p.resize(m->nverts);
            m->uv.resize(2 * (size_t)m->nverts);
            for (int y = 0, pos = 0; y < nv; ++y)
                for (int x = 0; x < nu; ++x, ++pos) {
                    const float px = (float)x / (float)(nu - 1), py = (float)y / (float)(nv - 1);
                    m->uv[2 * pos] = px; m->uv[2 * pos + 1] = py;
                    m->p[pos] = o2w.Point(V3(px, py, Pz->f[pos]));
                }
            m->vi.reserve(3 * (size_t)m->ntris);
            for (int y = 0; y < nv - 1; ++y)
                for (int x = 0; x < nu - 1; ++x) {
                    const int v00 = x + y * nu, v10 = (x + 1) + y * nu, v11 = (x + 1) + (y + 1) * nu, v01 = x + (y + 1) * nu;
                    m->vi.insert(m->vi.end(), {v00, v10, v11, v00, v11, v01});
                }
            s->kind = ShapeObj::HFIELD; s->mesh = m;
            allMeshes.push_back(m);
        } else if (name == "nurbs") {   // nurbs.cpp:221-298 Refine (30 x 30 dicing), 300-349 parameters
            const int nu = p.FindOneInt("nu", -1), uorder = p.FindOneInt("uorder", -1);
            const int nv = p.FindOneInt("nv", -1), vorder = p.FindOneInt("vorder", -1);
            const Param *uk = p.Find(P_FLOAT, "uknots"), *vk = p.Find(P_FLOAT, "vknots");
            if (nu < 1 || uorder < 2 || nv < 1 || vorder < 2 || !uk || !vk || (int)uk->f.size() != nu + uorder ||
                (int)vk->f.size() != nv + vorder)
                throw std::runtime_error("nurbs: nu / uorder / uknots and nv / vorder / vknots required");
            const float u0 = p.FindOneFloat("u0", uk->f[uorder - 1]), u1 = p.FindOneFloat("u1", uk->f[nu]);
            const float v0 = p.FindOneFloat("v0", vk->f[vorder - 1]), v1 = p.FindOneFloat("v1", vk->f[nv]);
            std::vector<NurbsH3> Pw((size_t)nu * nv);
            if (const Param *P = p.Find(P_POINT, "P")) {
                if ((int)P->f.size() / 3 != nu * nv) { out->warnings.push_back("NURBS shape: control point count"); return nullptr; }
                for (int i = 0; i < nu * nv; ++i) { Pw[i].x = P->f[3 * i]; Pw[i].y = P->f[3 * i + 1]; Pw[i].z = P->f[3 * i + 2]; Pw[i].w = 1.; }
            } else if (const Param *Q = p.Find(P_FLOAT, "Pw")) {
                if (Q->f.size() % 4 || (int)Q->f.size() / 4 != nu * nv) { out->warnings.push_back("NURBS shape: \"Pw\" count"); return nullptr; }
                for (int i = 0; i < nu * nv; ++i) { Pw[i].x = Q->f[4 * i]; Pw[i].y = Q->f[4 * i + 1]; Pw[i].z = Q->f[4 * i + 2]; Pw[i].w = Q->f[4 * i + 3]; }
            } else { out->warnings.push_back("Must provide control points via \"P\" or \"Pw\" parameter to NURBS shape."); return nullptr; }
            const int dice = 30;
            float ueval[dice], veval[dice];
            for (int i = 0; i < dice; ++i) ueval[i] = Lerp((float)i / (float)(dice - 1), u0, u1);
            for (int i = 0; i < dice; ++i) veval[i] = Lerp((float)i / (float)(dice - 1), v0, v1);
            auto m = std::make_shared<TriMesh>();
            m->o2w = o2w; m->ro = ro; m->swaps = o2w.SwapsHandedness();
            m->nverts = dice * dice; m->ntris = 2 * (dice - 1) * (dice - 1);
            m->p.resize(m->nverts); m->n.resize(m->nverts); m->uv.resize(2 * (size_t)m->nverts);
            for (int v = 0; v < dice; ++v)
                for (int u = 0; u < dice; ++u) {
                    const int k = v * dice + u;
                    m->uv[2 * k] = ueval[u]; m->uv[2 * k + 1] = veval[v];
                    V3 dPdu, dPdv;
                    const V3 pt = NurbsEvaluateSurface(uorder, uk->f.data(), nu, ueval[u], vorder, vk->f.data(), nv, veval[v],
                                                       Pw.data(), &dPdu, &dPdv);
                    m->p[k] = o2w.Point(pt);
                    m->n[k] = Normalize(Cross(dPdu, dPdv));
                }
            m->vi.reserve(3 * (size_t)m->ntris);
            for (int v = 0; v < dice - 1; ++v)
                for (int u = 0; u < dice - 1; ++u) {
                    const int a = v * dice + u, b = v * dice + u + 1, c2 = (v + 1) * dice + u + 1, d = (v + 1) * dice + u;
                    m->vi.insert(m->vi.end(), {a, b, c2, a, c2, d});
                }
            s->kind = ShapeObj::HFIELD; s->mesh = m;   // refined into one TriangleMesh, as a heightfield
            allMeshes.push_back(m);
        } else if (name == "loopsubdiv") {   // loopsubdiv.cpp:489-502
            int nlevels = p.FindOneInt("nlevels", 3);
            const Param *vi = p.Find(P_INT, "indices"), *P = p.Find(P_POINT, "P");
            if (!vi || !P) return nullptr;
            std::vector<V3> pts(P->f.size() / 3);
            for (size_t i = 0; i < pts.size(); ++i) pts[i] = V3(P->f[3 * i], P->f[3 * i + 1], P->f[3 * i + 2]);
            s->kind = ShapeObj::LOOP; s->o2w = o2w; s->ro = ro; s->nLevels = nlevels;
            LoopInit(*s, (int)vi->i.size() / 3, (int)pts.size(), vi->i.data(), pts.data());
        } else if (name == "sphere" || name == "disk" || name == "cylinder") {
            auto q = std::make_shared<Quadric>();
            q->o2w = o2w;
            pbrtgpu_quadric &Q = q->q;
            Q.reverse_orientation = ro; Q.swaps_handedness = o2w.SwapsHandedness();
            memcpy(Q.o2w_m, o2w.m.m, 64); memcpy(Q.o2w_minv, o2w.mInv.m, 64);
            if (name == "sphere") {   // sphere.cpp:33-43, 205-214
                float radius = p.FindOneFloat("radius", 1.f);
                float z0 = p.FindOneFloat("zmin", -radius), z1 = p.FindOneFloat("zmax", radius);
                float pm = p.FindOneFloat("phimax", 360.f);
                Q.type = PBRTGPU_SHAPE_SPHERE;
                Q.radius = radius;
                Q.zmin = Clamp(pmin(z0, z1), -radius, radius);
                Q.zmax = Clamp(pmax(z0, z1), -radius, radius);
                Q.theta_min = acosf(Clamp(Q.zmin / radius, -1.f, 1.f));
                Q.theta_max = acosf(Clamp(Q.zmax / radius, -1.f, 1.f));
                Q.phi_max = Radians(Clamp(pm, 0.0f, 360.0f));
            } else if (name == "cylinder") {   // cylinder.cpp:30-37, 184-192
                const float radius = p.FindOneFloat("radius", 1), z0 = p.FindOneFloat("zmin", -1), z1 = p.FindOneFloat("zmax", 1);
                Q.type = PBRTGPU_SHAPE_CYLINDER;
                Q.radius = radius;
                Q.zmin = pmin(z0, z1);
                Q.zmax = pmax(z0, z1);
                Q.phi_max = Radians(Clamp(p.FindOneFloat("phimax", 360), 0.0f, 360.0f));
            } else {   // disk.cpp:32-38, 125-131
                Q.type = PBRTGPU_SHAPE_DISK;
                Q.height = p.FindOneFloat("height", 0.);
                Q.radius = p.FindOneFloat("radius", 1);
                Q.inner_radius = p.FindOneFloat("innerradius", 0);
                Q.phi_max = Radians(Clamp(p.FindOneFloat("phimax", 360), 0.0f, 360.0f));
            }
            s->kind = ShapeObj::QUADRIC; s->quad = q;
            allQuads.push_back(q);
        } else
            throw std::runtime_error("shape '" + name + "' is not supported by this build yet");
        return s;
    }
    // Shape::Refine result in order (triangles 0..n-1 of the mesh)
    void RefineShape(const std::shared_ptr<ShapeObj> &s, std::vector<Isect> *outv) {
        if (s->kind == ShapeObj::QUADRIC) { Isect is; is.kind = s->quad->q.type; is.quad = s->quad.get(); outv->push_back(is); return; }
        TriMesh *m;
        if (s->kind == ShapeObj::LOOP) {
            if (!s->refined) { s->refined = LoopRefine(*s); allMeshes.push_back(s->refined); }
            m = s->refined.get();
        } else m = s->mesh.get();
        for (int i = 0; i < m->ntris; ++i) { Isect is; is.kind = PBRTGPU_SHAPE_TRIANGLE; is.mesh = m; is.tri = i; outv->push_back(is); }
    }
    void MakeShapeDirective(const std::string &name, const ParamSet &params) {   // api.cpp:1051-1123
        if (curT.IsAnimated()) {
            // api.cpp:1088-1118: shape built with the identity transform, refined, nested
            // BVH (default maxPrims 1) if more than one primitive, TransformedPrimitive with
            // the animated world->object transform
            if (gs.areaLight != "") out->warnings.push_back("Ignoring currently set area light when creating animated shape");
            Xform id, idInv;
            LookupCache(Xform(), &id, &idInv);
            auto shape = MakeShape(name, id, idInv, gs.reverseOrientation, params);
            if (!shape) return;
            auto mtl = CreateMaterialFromState(params);
            // api.cpp:1094-1105: GeometricPrimitive, its FullyRefine (one GeometricPrimitive per
            // refined shape: a mesh's triangles, a subdivision surface's mesh and then its
            // triangles), a BVHAccel over more than one, then the TransformedPrimitive
            nextPrimId++;
            if (shape->kind != ShapeObj::QUADRIC) {
                std::vector<Isect> r;
                RefineShape(shape, &r);
                nextPrimId += (uint32_t)r.size() + (shape->kind == ShapeObj::LOOP || shape->kind == ShapeObj::HFIELD ? 1u : 0u);
                if (r.empty()) return;   // api.cpp:1099: no TransformedPrimitive (and no id) then
                if (r.size() > 1) nextPrimId++;
            }
            Xform w2o0, w2o1;
            LookupCache(curT.t[0], nullptr, &w2o0);
            LookupCache(curT.t[1], nullptr, &w2o1);
            InstanceObj io;
            io.shape = shape; io.mtl = mtl;
            io.anim = AnimXform(w2o0, tStart, w2o1, tEnd);
            instanceObjs.push_back(io);
            PrimObj po; po.instance = (int)instanceObjs.size() - 1;
            po.refId = nextPrimId++;
            po.name = name;
            primitives.push_back(po);
            return;
        }
        Xform o2w, w2o;
        LookupCache(curT.t[0], &o2w, &w2o);
        auto shape = MakeShape(name, o2w, w2o, gs.reverseOrientation, params);
        if (!shape) return;
        auto mtl = CreateMaterialFromState(params);
        int area = -1;
        std::shared_ptr<LightObj> alo;
        if (gs.areaLight != "") {
            if (gs.areaLight != "area" && gs.areaLight != "diffuse")
                throw std::runtime_error("area light '" + gs.areaLight + "' unknown");
            // diffuse.cpp:50-58 : Lemit = L * scale, ShapeSet(shape)
            alo = std::make_shared<LightObj>();
            alo->l.type = PBRTGPU_LIGHT_AREA;
            Spec L = gs.areaLightParams.FindOneSpectrum("L", spec.Const(1.0f));
            Spec sc = gs.areaLightParams.FindOneSpectrum("scale", spec.Const(1.0f));
            alo->L = SpecMul(L, sc);
            alo->l.is_black = SpecIsBlack(alo->L);
            alo->l.n_samples = std::max(1, gs.areaLightParams.FindOneInt("nsamples", 1));   // diffuse.cpp:55
            ShapeSetOf(shape, &alo->shapeSet);
            Xform l2w = curT.t[0];
            memcpy(alo->l.l2w_m, l2w.m.m, 64); memcpy(alo->l.l2w_minv, l2w.mInv.m, 64);
        }
        PrimObj po; po.shape = shape; po.mtl = mtl;
        po.refId = nextPrimId++;   // api.cpp:1070 GeometricPrimitive
        po.name = name;
        if (alo) { lights.push_back(alo); po.areaLight = (int)lights.size() - 1; }
        primitives.push_back(po);
    }

    // ------------------------------ WorldEnd ---------------------------------------
    struct BuildPrim { Isect is; int material; int areaLight; uint32_t primId = 0, matId = 0; };
    struct PrimInfo { int primitiveNumber; V3 centroid; BBox bounds; };
    struct BuildNode { BBox bounds; int children[2] = {-1, -1}; uint32_t splitAxis = 0, firstPrimOffset = 0, nPrimitives = 0; };
    struct InstanceObj {
        std::shared_ptr<ShapeObj> shape;
        std::shared_ptr<MaterialObj> mtl;
        AnimXform anim;
    };
    std::vector<InstanceObj> instanceObjs;
    // one BVHAccel build (bvh.cpp:145-351): input prims in FullyRefine order -> nodes, ordered prims
    struct BvhBuild {
        uint32_t maxPrimsInNode = 4;
        std::vector<BuildNode> bnodes;
        std::vector<BuildPrim> prims, ordered;
        int maxDepth = 0;
        void Build() {
            std::vector<PrimInfo> bd(prims.size());
            for (size_t i = 0; i < prims.size(); ++i) {
                bd[i].primitiveNumber = (int)i;
                bd[i].bounds = prims[i].is.WorldBound();
                bd[i].centroid = .5f * bd[i].bounds.pMin + .5f * bd[i].bounds.pMax;
            }
            Recursive(bd, 0, (uint32_t)bd.size(), 0);
        }
            int Recursive(std::vector<PrimInfo> &bd, uint32_t start, uint32_t end, int depth) {   // bvh.cpp:202-351
            maxDepth = std::max(maxDepth, depth);
            int nodeIdx = (int)bnodes.size();
            bnodes.push_back(BuildNode());
            BBox bbox;
            for (uint32_t i = start; i < end; ++i) bbox = Union(bbox, bd[i].bounds);
            uint32_t nPrimitives = end - start;
            auto makeLeaf = [&]() {
                uint32_t first = (uint32_t)ordered.size();
                for (uint32_t i = start; i < end; ++i) ordered.push_back(prims[bd[i].primitiveNumber]);
                bnodes[nodeIdx].firstPrimOffset = first; bnodes[nodeIdx].nPrimitives = nPrimitives; bnodes[nodeIdx].bounds = bbox;
                return nodeIdx;
            };
            if (nPrimitives == 1) return makeLeaf();
            BBox cb;
            for (uint32_t i = start; i < end; ++i) cb = Union(cb, bd[i].centroid);
            int dim = cb.MaximumExtent();
            uint32_t mid = (start + end) / 2;
            if (cb.pMax[dim] == cb.pMin[dim]) return makeLeaf();
            auto cmpPts = [dim](const PrimInfo &a, const PrimInfo &b) { return a.centroid[dim] < b.centroid[dim]; };
            if (nPrimitives <= 4) {
                mid = (start + end) / 2;
                std::nth_element(&bd[start], &bd[mid], &bd[end - 1] + 1, cmpPts);
            } else {
                const int nBuckets = 12;
                struct Bucket { int count = 0; BBox bounds; } buckets[nBuckets];
                for (uint32_t i = start; i < end; ++i) {
                    int b = nBuckets * ((bd[i].centroid[dim] - cb.pMin[dim]) / (cb.pMax[dim] - cb.pMin[dim]));
                    if (b == nBuckets) b = nBuckets - 1;
                    buckets[b].count++;
                    buckets[b].bounds = Union(buckets[b].bounds, bd[i].bounds);
                }
                float cost[nBuckets - 1];
                for (int i = 0; i < nBuckets - 1; ++i) {
                    BBox b0, b1;
                    int count0 = 0, count1 = 0;
                    for (int j = 0; j <= i; ++j) { b0 = Union(b0, buckets[j].bounds); count0 += buckets[j].count; }
                    for (int j = i + 1; j < nBuckets; ++j) { b1 = Union(b1, buckets[j].bounds); count1 += buckets[j].count; }
                    cost[i] = .125f + (count0 * b0.SurfaceArea() + count1 * b1.SurfaceArea()) / bbox.SurfaceArea();
                }
                float minCost = cost[0];
                uint32_t minCostSplit = 0;
                for (int i = 1; i < nBuckets - 1; ++i)
                    if (cost[i] < minCost) { minCost = cost[i]; minCostSplit = i; }
                if (nPrimitives > maxPrimsInNode || minCost < nPrimitives) {
                    float pmin_ = cb.pMin[dim], pmax_ = cb.pMax[dim];
                    int splitBucket = (int)minCostSplit;   // CompareToBucket (bvh.cpp:84-101)
                    PrimInfo *pm = std::partition(&bd[start], &bd[end - 1] + 1, [&](const PrimInfo &p) {
                        int b = nBuckets * ((p.centroid[dim] - pmin_) / (pmax_ - pmin_));
                        if (b == nBuckets) b = nBuckets - 1;
                        return b <= splitBucket;
                    });
                    mid = (uint32_t)(pm - &bd[0]);
                } else
                    return makeLeaf();
            }
            int c0 = Recursive(bd, start, mid, depth + 1);
            int c1 = Recursive(bd, mid, end, depth + 1);
            BuildNode &n = bnodes[nodeIdx];
            n.children[0] = c0; n.children[1] = c1;
            n.bounds = Union(bnodes[c0].bounds, bnodes[c1].bounds);
            n.splitAxis = dim; n.nPrimitives = 0;
            return nodeIdx;
        }
    };
    BvhBuild top;
    std::vector<BvhBuild> blas;   // per instance (no nodes if the instance is a single primitive)

    // bvh.cpp:354-372; nodes go to out->nodes from *offset, leaf prim offsets are shifted by
    // primBase (prims of all BVHs share one array)
    uint32_t Flatten(const BvhBuild &B, int node, uint32_t *offset, uint32_t primBase) {
        pbrtgpu_bvh_node &ln = out->nodes[*offset];
        const BuildNode &bn = B.bnodes[node];
        for (int k = 0; k < 3; ++k) { ln.bmin[k] = bn.bounds.pMin[k]; ln.bmax[k] = bn.bounds.pMax[k]; }
        uint32_t my = (*offset)++;
        if (bn.nPrimitives > 0) {
            ln.offset = primBase + bn.firstPrimOffset;
            ln.meta = bn.nPrimitives & 0xff;
        } else {
            out->nodes[my].meta = (bn.splitAxis & 0xff) << 8;
            Flatten(B, bn.children[0], offset, primBase);
            uint32_t second = Flatten(B, bn.children[1], offset, primBase);
            out->nodes[my].offset = second;
        }
        return my;
    }
    void EmitPrims(const std::vector<BuildPrim> &v, int inst) {
        for (auto &bp : v) {
            pbrtgpu_prim fp;
            if (bp.is.kind == PBRTGPU_SHAPE_INSTANCE) { fp.shape_type = PBRTGPU_SHAPE_INSTANCE; fp.shape_index = bp.is.inst; }
            else fp.shape_index = EmitShape(bp.is, &fp.shape_type);
            fp.material = bp.material;
            fp.area_light = bp.areaLight;
            out->prims.push_back(fp);
            out->primInstance.push_back(inst);
            out->primMeta.push_back(bp.primId);
            out->primMeta.push_back(bp.matId);
        }
    }

    int EmitMesh(TriMesh *m) {
        if (m->flatIndex >= 0) return m->flatIndex;
        pbrtgpu_mesh fm{};
        memcpy(fm.o2w_m, m->o2w.m.m, 64); memcpy(fm.o2w_minv, m->o2w.mInv.m, 64);
        fm.has_normals = !m->n.empty(); fm.has_uvs = !m->uv.empty();
        fm.reverse_orientation = m->ro; fm.swaps_handedness = m->swaps;
        fm.vert_offset = (int)(out->vertP.size() / 3); fm.nverts = m->nverts;
        for (int i = 0; i < m->nverts; ++i) {
            out->vertP.push_back(m->p[i].x); out->vertP.push_back(m->p[i].y); out->vertP.push_back(m->p[i].z);
            V3 n = m->n.empty() ? V3() : m->n[i];
            out->vertN.push_back(n.x); out->vertN.push_back(n.y); out->vertN.push_back(n.z);
            out->vertUV.push_back(m->uv.empty() ? 0.f : m->uv[2 * i]);
            out->vertUV.push_back(m->uv.empty() ? 0.f : m->uv[2 * i + 1]);
        }
        out->meshes.push_back(fm);
        m->flatIndex = (int)out->meshes.size() - 1;
        return m->flatIndex;
    }
    int EmitShape(const Isect &is, int *type) {
        *type = is.kind;
        if (is.kind == PBRTGPU_SHAPE_TRIANGLE) {
            int mi = EmitMesh(is.mesh);
            pbrtgpu_triangle t;
            t.mesh = mi;
            int off = out->meshes[mi].vert_offset;
            for (int k = 0; k < 3; ++k) t.v[k] = is.mesh->vi[3 * is.tri + k] + off;
            out->tris.push_back(t);
            return (int)out->tris.size() - 1;
        }
        if (is.quad->flatIndex < 0) { out->quadrics.push_back(is.quad->q); is.quad->flatIndex = (int)out->quadrics.size() - 1; }
        return is.quad->flatIndex;
    }
    int EmitSpectrum(const Spec &s) {
        int off = (int)out->spectra.size();
        out->spectra.insert(out->spectra.end(), s.begin(), s.end());
        return off;
    }
    int EmitMaterial(MaterialObj *m) {
        if (m->flatIndex >= 0) return m->flatIndex;
        pbrtgpu_material fm = m->m;
        for (int k = 0; k < 4; ++k) fm.spec[k] = k < (int)m->spectra.size() ? EmitSpectrum(m->spectra[k]) : -1;
        fm.black_mask &= ~0xf;   // bits 4-7 (unclamped textured slots) stay
        for (int k = 0; k < (int)m->spectra.size() && k < 4; ++k)
            if (fm.tex[k] < 0 && SpecIsBlack(m->spectra[k])) fm.black_mask |= 1 << k;
        if (m->measured) fm.aux = EmitMeasured(m->measured.get(), &fm.aux2);
        out->materials.push_back(fm);
        m->flatIndex = (int)out->materials.size() - 1;
        return m->flatIndex;
    }

    // CreateRealisticDiffractionCamera + the constructor's lens file (realisticDiffraction.cpp:
    // 32-193): shutter times default to -1 (not swapped); the lens file is ReadFloatFile's
    // floats, the focal length then (radius, separation, n, aperture) per element, an aperture
    // stop (radius 0) taking "aperture_diameter"; "diffractionEnabled" (on by default) is
    // GenerateRay's Gaussian perturbation per element.  The light-field modes: "num_pinholes_w/h"
    // (ints of float parameters, :73-75) a pinhole array whose positions Flat() computes at the film
    // resolution, "microlens_enabled" (FindOneFloat, :76) a microlens per pinhole; "IORforEyeEnabled"
    // (:82) the Gullstrand eye's IOR spectra (FromSampled of its curves, :196-205; eye_ior_tables.inc).
    void RealisticCamera(CameraParams *cp) {
        const ParamSet &p = cameraParams;
        cp->shutterOpen = p.FindOneFloat("shutteropen", -1.f);
        cp->shutterClose = p.FindOneFloat("shutterclose", -1.f);
        std::string spec = p.FindOneString("specfile", "");
        if (spec.empty()) throw std::runtime_error("No lens spec file supplied!");
        pbrtgpu_lens &L = out->lens;
        memset(&L, 0, sizeof(L));
        L.num_pinholes_w = (int)p.FindOneFloat("num_pinholes_w", -1);
        L.num_pinholes_h = (int)p.FindOneFloat("num_pinholes_h", -1);
        L.microlens = p.FindOneFloat("microlens_enabled", 0) != 0 ? 1 : 0;
        L.ior_eye = p.FindOneBool("IORforEyeEnabled", false) ? 1 : 0;
        out->eyeIor.clear();
        if (L.ior_eye) {
            const float(*t)[32] = nullptr;
            const float(*t60)[60] = nullptr;
            const float(*t30)[30] = nullptr;
            if (ov.bands == 32) t = kEyeIor_32_395_715;
            else if (ov.bands == 60) t60 = kEyeIor_60_395_715;
            else if (ov.bands == 30) t30 = kEyeIor_30_400_700;
            else throw std::runtime_error("realisticDiffraction: IORforEyeEnabled needs SampledSpectrum (30, 32 or 60 bands)");
            for (int k = 0; k < 4; ++k)
                for (int i = 0; i < ov.bands; ++i) out->eyeIor.push_back(t ? t[k][i] : t60 ? t60[k][i] : t30[k][i]);
        }
        L.chromatic = p.FindOneBool("chromaticAberrationEnabled", false) ? 1 : 0;
        L.diffraction = p.FindOneBool("diffractionEnabled", true) ? 1 : 0;   // realisticDiffraction.cpp:61,128
        L.film_distance = p.FindOneFloat("filmdistance", 70.f);
        const float apDiam = p.FindOneFloat("aperture_diameter", 1.f);
        L.film_diag = p.FindOneFloat("filmdiag", 35.f);
        L.curve_radius = p.FindOneFloat("curveRadius", 0.f);
        L.aperture_offset[0] = p.FindOneFloat("x_aperture_offset", 0.f);
        L.aperture_offset[1] = p.FindOneFloat("y_aperture_offset", 0.f);
        L.film_center[0] = p.FindOneFloat("film_center_x", 0.f);
        L.film_center[1] = p.FindOneFloat("film_center_y", 0.f);
        L.pinhole_exit[0] = p.FindOneFloat("pinhole_exit_x", -1.f);
        L.pinhole_exit[1] = p.FindOneFloat("pinhole_exit_y", -1.f);
        L.pinhole_exit[2] = p.FindOneFloat("pinhole_exit_z", -1.f);
        std::vector<float> vals = ReadFloatFile(Resolve(spec));
        if (vals.empty()) throw std::runtime_error("Unable to read lens file " + spec);
        if ((vals.size() - 1) % 4 != 0) throw std::runtime_error("Wrong number of float values in lens file " + spec);
        L.focal_length = vals[0];
        L.fstop = L.focal_length / apDiam;
        out->lensEl.clear();
        for (size_t i = 1; i < vals.size(); i += 4) {
            float el[4] = {vals[i], vals[i + 1], vals[i + 2], vals[i + 3]};
            if (el[0] == 0) el[3] = apDiam;
            out->lensEl.insert(out->lensEl.end(), el, el + 4);
        }
        const int n = (int)out->lensEl.size() / 4;
        if (n == 0) throw std::runtime_error("lens file " + spec + " has no elements");
        // GenerateRay reads lensEls[i - 2].n when element i - 1 has n == 0 (realisticDiffraction.cpp:960-966)
        if (n >= 2 && out->lensEl[2] == 0 && out->lensEl[4] != 0)
            throw std::runtime_error("lens file " + spec + ": element 0 has n == 0");
        if (L.num_pinholes_w > 0 && L.num_pinholes_h > 0 && (size_t)L.num_pinholes_w * L.num_pinholes_h > (1u << 24))
            throw std::runtime_error("realisticDiffraction: pinhole array too large");
        out->cameraType = PBRTGPU_CAMERA_REALISTIC;
    }

    void WorldEnd() {
        while (!pushedGS.empty()) { gs = pushedGS.back(); pushedGS.pop_back(); }
        // ---- film (spectralImage.cpp:452-475) and sample extent (176-185)
        int xres = ov.xres > 0 ? ov.xres : filmParams.FindOneInt("xresolution", 640);
        int yres = ov.yres > 0 ? ov.yres : filmParams.FindOneInt("yresolution", 480);
        float crop[4] = {0, 1, 0, 1};
        const Param *cr = filmParams.Find(P_FLOAT, "cropwindow");
        if (cr && cr->f.size() == 4) {
            crop[0] = Clamp(pmin(cr->f[0], cr->f[1]), 0., 1.); crop[1] = Clamp(pmax(cr->f[0], cr->f[1]), 0., 1.);
            crop[2] = Clamp(pmin(cr->f[2], cr->f[3]), 0., 1.); crop[3] = Clamp(pmax(cr->f[2], cr->f[3]), 0., 1.);
        }
        // ---- camera (perspective.cpp:110-147, orthographic.cpp:105-140) -- parameters kept
        // resolution independent
        if (cameraName != "perspective" && cameraName != "orthographic" && cameraName != "realisticDiffraction")
            throw std::runtime_error("camera '" + cameraName + "' is not supported by this build");
        Xform c2w[2];
        for (int i = 0; i < 2; ++i) LookupCache(cameraToWorld.t[i], &c2w[i], nullptr);
        // an animated CameraToWorld (AnimatedTransform(cam2world[0], transformStartTime,
        // cam2world[1], transformEndTime), api.cpp MakeCamera): its start / end matrices and
        // Decompose for the per-ray Interpolate (camera.cpp:84-103)
        out->cameraMotion.clear();
        if (c2w[0] != c2w[1]) {
            const AnimXform A(c2w[0], tStart, c2w[1], tEnd);
            pbrtgpu_instance cm{};
            cm.root = -1; cm.single_prim = -1;
            cm.animated = A.animated ? 1 : 0;
            cm.start_time = A.startTime; cm.end_time = A.endTime;
            memcpy(cm.start_m, A.start.m.m, 64); memcpy(cm.start_minv, A.start.mInv.m, 64);
            memcpy(cm.end_m, A.end.m.m, 64); memcpy(cm.end_minv, A.end.mInv.m, 64);
            for (int k = 0; k < 2; ++k) {
                cm.T[k][0] = A.T[k].x; cm.T[k][1] = A.T[k].y; cm.T[k][2] = A.T[k].z; cm.T[k][3] = 0.f;
                cm.R[k][0] = A.R[k].v.x; cm.R[k][1] = A.R[k].v.y; cm.R[k][2] = A.R[k].v.z; cm.R[k][3] = A.R[k].w;
                memcpy(cm.S[k], A.S[k].m, 64);
            }
            out->cameraMotion.push_back(cm);
        }
        CameraParams &cp = out->camParams;
        cp.shutterOpen = cameraParams.FindOneFloat("shutteropen", 0.f);
        cp.shutterClose = cameraParams.FindOneFloat("shutterclose", 1.f);
        if (cp.shutterClose < cp.shutterOpen) std::swap(cp.shutterOpen, cp.shutterClose);
        out->cameraType = cameraName == "orthographic" ? PBRTGPU_CAMERA_ORTHOGRAPHIC : PBRTGPU_CAMERA_PERSPECTIVE;
        if (cameraName == "realisticDiffraction") RealisticCamera(&cp);
        cp.lensRadius = cameraParams.FindOneFloat("lensradius", 0.f);
        cp.focalDistance = cameraParams.FindOneFloat("focaldistance", 1e30f);
        const Param *fa = cameraParams.Find(P_FLOAT, "frameaspectratio");
        cp.hasFrameAspect = fa && fa->f.size();
        cp.frameAspect = cp.hasFrameAspect ? fa->f[0] : 0.f;
        const Param *sw = cameraParams.Find(P_FLOAT, "screenwindow");
        cp.hasScreenWindow = sw && sw->f.size() == 4;
        if (cp.hasScreenWindow) for (int k = 0; k < 4; ++k) cp.screenWindow[k] = sw->f[k];
        cp.fov = cameraParams.FindOneFloat("fov", 90.);
        float halffov = cameraParams.FindOneFloat("halffov", -1.f);
        if (halffov > 0.f) cp.fov = 2.f * halffov;
        for (int k = 0; k < 4; ++k) cp.crop[k] = crop[k];
        memcpy(cp.cam2world, c2w[0].m.m, 64);
        cp.xres = xres; cp.yres = yres;
        ComputeCamera(cp, xres, yres, &out->camera, out->cameraType);
        // ---- integrator / sampler
        out->maxDepth = ov.maxdepth >= 0 ? ov.maxdepth : surfParams.FindOneInt("maxdepth", 5);
        // SurfaceIntegrator (api.cpp:551-583): "path" or "directlighting" (strategy "all" / "one",
        // unknown strategies -> "all" with a warning, directlighting.cpp:115-125); others are
        // rejected rather than rendered as something else
        if (ov.integrator >= 0) out->integrator = ov.integrator;
        else if (surfName == "path") out->integrator = PBRTGPU_INTEGRATOR_PATH;
        else if (surfName == "directlighting") out->integrator = PBRTGPU_INTEGRATOR_DIRECT;
        else if (surfName == "metadata") out->integrator = PBRTGPU_INTEGRATOR_METADATA;
        else throw std::runtime_error("SurfaceIntegrator '" + surfName + "' is not supported by this build");
        out->surfStrategy = surfParams.FindOneString("strategy", "");
        std::string st = surfParams.FindOneString("strategy", "all");
        if (out->integrator == PBRTGPU_INTEGRATOR_DIRECT && st != "all" && st != "one")
            out->warnings.push_back("Strategy \"" + st + "\" for direct lighting unknown");
        out->dlStrategy = ov.dl_strategy >= 0 ? ov.dl_strategy : (st == "one" ? PBRTGPU_DL_ONE : PBRTGPU_DL_ALL);
        // CreateMetadataIntegrator (metadata.cpp:83-97): "mesh", "material", "depth" (default;
        // unknown strategies -> "depth" with a warning)
        std::string ms = surfParams.FindOneString("strategy", "depth");
        out->metaStrategy = ms == "mesh" ? PBRTGPU_META_MESH : ms == "material" ? PBRTGPU_META_MATERIAL : PBRTGPU_META_DEPTH;
        if (out->integrator == PBRTGPU_INTEGRATOR_METADATA && ms != "mesh" && ms != "material" && ms != "depth")
            out->warnings.push_back("Strategy \"" + ms + "\" for metadata unknown");
        if (ov.meta_strategy >= 0) out->metaStrategy = ov.meta_strategy;
        // Renderer (api.cpp:1369-1407): "spectralrenderer" with "nWaveBands" (default 32) and
        // "samplingMethod" ("singleDirection" default, or "samplerDirection"); every other
        // name renders as "sampler" (the configs override "metropolis")
        out->renderer = PBRTGPU_RENDERER_SAMPLER;
        if (rendererName == "spectralrenderer") {
            out->renderer = PBRTGPU_RENDERER_SPECTRAL;
            out->waveBands = rendererParams.FindOneInt("nWaveBands", 32);
            std::string sm = rendererParams.FindOneString("samplingMethod", "singleDirection");
            if (sm == "singleDirection") out->spectralSampling = PBRTGPU_SPECTRAL_SINGLE;
            else if (sm == "samplerDirection") out->spectralSampling = PBRTGPU_SPECTRAL_SAMPLER;
            else throw std::runtime_error("Unrecognized spectral sampling method \"" + sm + "\"");
        }
        if (ov.renderer >= 0) out->renderer = ov.renderer;
        if (ov.wave_bands > 0) out->waveBands = ov.wave_bands;
        if (ov.spectral_sampling >= 0) out->spectralSampling = ov.spectral_sampling;
        int nsamp = ov.spp > 0 ? ov.spp : samplerParams.FindOneInt("pixelsamples", 4);
        out->spp = (int)RoundUpPow2((uint32_t)nsamp);
        out->seed = ov.seed == 0xffffffffu ? 0u : ov.seed;   // PBRTHOST_KEEP_SEED
        out->nBands = spec.n();
        out->bandY.assign(spec.Y(), spec.Y() + spec.n());
        out->yint = spec.yint();
        // ---- refine primitives (primitive.cpp:40-53, LIFO) and build the BVHs
        // ids: hits on a top-level primitive report its refined GeometricPrimitive's id (created
        // in triangle order by Refine, primitive.cpp:137-148, after the subdivision mesh's own);
        // hits inside a TransformedPrimitive report the TransformedPrimitive's (primitive.cpp:95)
        auto refineInto = [&](const std::shared_ptr<ShapeObj> &shape, MaterialObj *mtl, int areaLight,
                              uint32_t fixedId, std::vector<BuildPrim> *dst) {
            std::vector<Isect> r;
            RefineShape(shape, &r);
            uint32_t base = fixedId;
            if (!fixedId) {
                if (shape->kind == ShapeObj::LOOP || shape->kind == ShapeObj::HFIELD) nextPrimId++;   // the refined mesh's own
                base = nextPrimId;
                nextPrimId += (uint32_t)r.size();
            }
            // single intersectable shape -> itself; refinable -> children popped in reverse
            for (size_t k = r.size(); k-- > 0;) {
                BuildPrim bp; bp.is = r[k]; bp.material = EmitMaterial(mtl); bp.areaLight = areaLight;
                bp.primId = fixedId ? fixedId : base + (uint32_t)k;
                bp.matId = mtl->refId;
                dst->push_back(bp);
            }
        };
        nextPrimId++;   // the scene's BVHAccel (MakeScene -> MakeAccelerator, api.cpp:1318)
        blas.assign(instanceObjs.size(), BvhBuild());
        for (auto &po : primitives) {
            if (po.instance < 0) {
                refineInto(po.shape, po.mtl.get(), po.areaLight, po.shape->kind == ShapeObj::QUADRIC ? po.refId : 0u,
                           &top.prims);
                continue;
            }
            // TransformedPrimitive (api.cpp:1101-1118): nested BVHAccel(refined) with the
            // default maxPrims 1, or the single refined primitive itself
            InstanceObj &io = instanceObjs[po.instance];
            BvhBuild &B = blas[po.instance];
            B.maxPrimsInNode = 1;
            refineInto(io.shape, io.mtl.get(), -1, po.refId, &B.prims);
            if (B.prims.empty()) continue;
            BBox objBound;
            if (B.prims.size() > 1) { B.Build(); objBound = B.bnodes[0].bounds; }
            else objBound = B.prims[0].is.WorldBound();
            BuildPrim tp;
            tp.is.kind = PBRTGPU_SHAPE_INSTANCE;
            tp.is.inst = po.instance;
            tp.is.instBound = io.anim.MotionBounds(objBound, true);   // TransformedPrimitive::WorldBound
            tp.material = -1; tp.areaLight = -1;
            tp.primId = po.refId; tp.matId = io.mtl->refId;
            top.prims.push_back(tp);
        }
        if (top.prims.empty()) throw std::runtime_error("scene has no primitives");
        // pbrtWorldEnd's metadata lists (api.cpp:1252-1276)
        for (auto &po : primitives) out->metaMesh.push_back(std::make_pair(po.refId, po.name));
        for (auto &nm : gs.namedMaterials)
            if (nm.second) out->metaMaterials.push_back(std::make_pair(nm.second->refId, nm.first));
        const auto tb0 = std::chrono::steady_clock::now();
        top.Build();
        if (getenv("PBRTHOST_TIMING"))
            fprintf(stderr, "pbrthost: parse+refine %.1f ms, top-level BVH build %.1f ms\n",
                    std::chrono::duration<double, std::milli>(tb0 - tLoad0).count(),
                    std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tb0).count());
        out->bvhMaxDepth = top.maxDepth;
        size_t nNodes = top.bnodes.size();
        for (auto &B : blas) nNodes += B.bnodes.size();
        out->nodes.assign(nNodes, pbrtgpu_bvh_node());
        uint32_t off = 0;
        Flatten(top, 0, &off, 0);
        EmitPrims(top.ordered, -1);
        for (size_t i = 0; i < instanceObjs.size(); ++i) {
            BvhBuild &B = blas[i];
            const InstanceObj &io = instanceObjs[i];
            pbrtgpu_instance fi{};
            fi.root = -1; fi.single_prim = -1;
            uint32_t primBase = (uint32_t)out->prims.size();
            if (B.prims.size() > 1) {
                fi.root = (int)off;
                Flatten(B, 0, &off, primBase);
                EmitPrims(B.ordered, (int)i);
                out->bvhMaxDepth = std::max(out->bvhMaxDepth, top.maxDepth + 1 + B.maxDepth);
            } else if (B.prims.size() == 1) {
                fi.single_prim = (int)primBase;
                EmitPrims(B.prims, (int)i);
            }
            const AnimXform &A = io.anim;
            fi.animated = A.animated ? 1 : 0;
            fi.start_time = A.startTime; fi.end_time = A.endTime;
            memcpy(fi.start_m, A.start.m.m, 64); memcpy(fi.start_minv, A.start.mInv.m, 64);
            memcpy(fi.end_m, A.end.m.m, 64); memcpy(fi.end_minv, A.end.mInv.m, 64);
            for (int k = 0; k < 2; ++k) {
                fi.T[k][0] = A.T[k].x; fi.T[k][1] = A.T[k].y; fi.T[k][2] = A.T[k].z; fi.T[k][3] = 0.f;
                fi.R[k][0] = A.R[k].v.x; fi.R[k][1] = A.R[k].v.y; fi.R[k][2] = A.R[k].v.z; fi.R[k][3] = A.R[k].w;
                memcpy(fi.S[k], A.S[k].m, 64);
            }
            out->instances.push_back(fi);
        }
        // ---- lights
        for (auto &lo : lights) {
            pbrtgpu_light fl = lo->l;
            fl.spec = EmitSpectrum(lo->L);
            if (fl.type == PBRTGPU_LIGHT_AREA) {
                fl.shape_offset = (int)out->lightShapes.size();
                fl.n_shapes = (int)lo->shapeSet.size();
                // ShapeSet areas + Distribution1D (montecarlo.h:46-66)
                std::vector<float> areas;
                float sumArea = 0.f;
                for (auto &is : lo->shapeSet) { float a = is.Area(); areas.push_back(a); sumArea += a; }
                int n = (int)areas.size();
                std::vector<float> cdf(n + 1);
                cdf[0] = 0.;
                for (int i = 1; i < n + 1; ++i) cdf[i] = cdf[i - 1] + areas[i - 1] / n;
                float funcInt = cdf[n];
                if (funcInt == 0.f) for (int i = 1; i < n + 1; ++i) cdf[i] = float(i) / float(n);
                else for (int i = 1; i < n + 1; ++i) cdf[i] /= funcInt;
                for (int i = 0; i < n; ++i) {
                    pbrtgpu_light_shape ls;
                    ls.shape_index = EmitShape(lo->shapeSet[i], &ls.shape_type);
                    ls.area = areas[i];
                    ls.cdf = cdf[i + 1];
                    out->lightShapes.push_back(ls);
                }
                fl.sum_area = sumArea;
            }
            out->lights.push_back(fl);
        }
        // ---- MIPMap::weightLut (mipmap.h:185-193) and the FromRGB basis tables
        out->ewaLut.resize(128);
        for (int i = 0; i < 128; ++i) {
            float alpha = 2;
            float r2 = float(i) / float(128 - 1);
            out->ewaLut[i] = expf(-alpha * r2) - expf(-alpha);
        }
        out->rgbBasis.clear();
        for (int k = 0; k < 14; ++k) out->rgbBasis.insert(out->rgbBasis.end(), spec.Basis(k), spec.Basis(k) + spec.n());
    }
};

// film extent (spectralImage.cpp:40-50, 176-185) and projective camera matrices
// (camera.cpp:84-103, perspective.cpp:33-40) for a film resolution
void ComputeCamera(const CameraParams &cp, int xres, int yres, pbrtgpu_camera *outc, int cameraType) {
    pbrtgpu_camera &C = *outc;
    memset(&C, 0, sizeof(C));
    C.xres = xres; C.yres = yres;
    C.px_start = Ceil2Int(xres * cp.crop[0]);
    C.px_count = std::max(1, Ceil2Int(xres * cp.crop[1]) - C.px_start);
    C.py_start = Ceil2Int(yres * cp.crop[2]);
    C.py_count = std::max(1, Ceil2Int(yres * cp.crop[3]) - C.py_start);
    const float fw = 0.5f;   // BoxFilter default width (box.cpp:36-41); other filters are refused at PixelFilter
    C.sx_start = Floor2Int(C.px_start + 0.5f - fw);
    C.sx_end = Floor2Int(C.px_start + 0.5f + C.px_count + fw);
    C.sy_start = Floor2Int(C.py_start + 0.5f - fw);
    C.sy_end = Floor2Int(C.py_start + 0.5f + C.py_count + fw);
    float frame = cp.hasFrameAspect ? cp.frameAspect : float(xres) / float(yres);
    float screen[4];
    if (frame > 1.f) { screen[0] = -frame; screen[1] = frame; screen[2] = -1.f; screen[3] = 1.f; }
    else { screen[0] = -1.f; screen[1] = 1.f; screen[2] = -1.f / frame; screen[3] = 1.f / frame; }
    if (cp.hasScreenWindow) for (int k = 0; k < 4; ++k) screen[k] = cp.screenWindow[k];
    const bool ortho = cameraType == PBRTGPU_CAMERA_ORTHOGRAPHIC;
    // CameraToScreen: Perspective(fov, 1e-2f, 1000.f) or Orthographic(0., 1.) (transform.cpp:292-295)
    Xform camToScreen = ortho ? Scale(1.f, 1.f, 1.f / (1.f - 0.f)) * Translate(V3(0.f, 0.f, -0.f))
                              : Perspective(cp.fov, 1e-2f, 1000.f);
    Xform screenToRaster = Scale(float(xres), float(yres), 1.f) *
                           Scale(1.f / (screen[1] - screen[0]), 1.f / (screen[2] - screen[3]), 1.f) *
                           Translate(V3(-screen[0], -screen[3], 0.f));
    Xform rasterToScreen = Inverse(screenToRaster);
    Xform rasterToCamera = Inverse(camToScreen) * rasterToScreen;
    memcpy(C.raster_to_camera, rasterToCamera.m.m, 64);
    // dxCamera / dyCamera: differences of raster points one pixel apart (perspective.cpp:45-48), or
    // the raster unit vectors themselves (orthographic.cpp:39-40)
    if (ortho) {
        const V3 dx = rasterToCamera.Vector(V3(1, 0, 0)), dy = rasterToCamera.Vector(V3(0, 1, 0));
        C.dx_camera[0] = dx.x; C.dx_camera[1] = dx.y; C.dx_camera[2] = dx.z;
        C.dy_camera[0] = dy.x; C.dy_camera[1] = dy.y; C.dy_camera[2] = dy.z;
        C.ortho = 1;
    } else {
        V3 r0 = rasterToCamera.Point(V3(0, 0, 0)), rx = rasterToCamera.Point(V3(1, 0, 0)), ry = rasterToCamera.Point(V3(0, 1, 0));
        C.dx_camera[0] = rx.x - r0.x; C.dx_camera[1] = rx.y - r0.y; C.dx_camera[2] = rx.z - r0.z;
        C.dy_camera[0] = ry.x - r0.x; C.dy_camera[1] = ry.y - r0.y; C.dy_camera[2] = ry.z - r0.z;
    }
    memcpy(C.cam2world_m, cp.cam2world, 64);
    C.lens_radius = cp.lensRadius; C.focal_distance = cp.focalDistance;
    C.shutter_open = cp.shutterOpen; C.shutter_close = cp.shutterClose;
}

bool LoadPbrtScene(const std::string &path, const RenderOverrides &ov, HostScene *out, std::string *err) {
    try {
        Builder b(path, ov, out);
        b.Run(path);
        return true;
    } catch (const std::exception &e) {
        if (err) *err = e.what();
        return false;
    }
}

void HostScene::Flat(pbrtgpu_flat_scene *f) const {
    memset(f, 0, sizeof(*f));
    f->abi_version = PBRTGPU_ABI_VERSION;
    f->n_bands = nBands; f->max_depth = maxDepth; f->spp = spp; f->seed = seed;
    f->y_int = yint; f->band_Y = bandY.data();
    f->camera = camera;
    f->n_nodes = (int)nodes.size(); f->nodes = nodes.data();
    f->n_prims = (int)prims.size(); f->prims = prims.data();
    f->n_tris = (int)tris.size(); f->tris = tris.data();
    f->n_meshes = (int)meshes.size(); f->meshes = meshes.data();
    f->n_verts = (int)(vertP.size() / 3); f->vert_p = vertP.data(); f->vert_n = vertN.data(); f->vert_uv = vertUV.data();
    f->n_quadrics = (int)quadrics.size(); f->quadrics = quadrics.data();
    f->n_materials = (int)materials.size(); f->materials = materials.data();
    f->n_lights = (int)lights.size(); f->lights = lights.data();
    f->n_light_shapes = (int)lightShapes.size(); f->light_shapes = lightShapes.data();
    f->n_spectra_floats = (int)spectra.size(); f->spectra = spectra.data();
    f->n_instances = (int)instances.size(); f->instances = instances.empty() ? nullptr : instances.data();
    f->prim_instance = primInstance.data();
    f->n_kdnodes = (int)kdnodes.size(); f->kdnodes = kdnodes.empty() ? nullptr : kdnodes.data();
    f->n_textures = (int)textures.size(); f->textures = textures.empty() ? nullptr : textures.data();
    f->ewa_lut = ewaLut.empty() ? nullptr : ewaLut.data();
    f->rgb_basis = rgbBasis.empty() ? nullptr : rgbBasis.data();
    f->n_merl_floats = (int)merl.size();
    f->merl = merl.empty() ? nullptr : merl.data();
    f->integrator = integrator;
    f->dl_strategy = dlStrategy;
    f->meta_strategy = metaStrategy;
    f->prim_meta = primMeta.size() == 2 * prims.size() && !prims.empty() ? primMeta.data() : nullptr;
    f->renderer = renderer;
    f->wave_bands = waveBands;
    f->spectral_sampling = spectralSampling;
    f->camera_type = cameraType;
    f->lens = lens;
    f->n_texel_floats = (int32_t)texels.size();
    f->texels = texels.empty() ? nullptr : texels.data();
    f->camera_motion = cameraMotion.empty() ? nullptr : cameraMotion.data();
    f->lens.n_elements = (int)lensEl.size() / 4;
    f->lens.elements = lensEl.empty() ? nullptr : lensEl.data();
    f->lens.eye_ior = lens.ior_eye && (int)eyeIor.size() == 4 * nBands ? eyeIor.data() : nullptr;
    f->lens.pinholes = nullptr;
    if (cameraType == PBRTGPU_CAMERA_REALISTIC && lens.num_pinholes_w > 0 && lens.num_pinholes_h > 0 && !lensEl.empty()) {
        // RealisticDiffractionCamera's pinhole array (realisticDiffraction.cpp:248-304), at the film
        // resolution the camera sees (getSensorWidth, :470-476): the superpixel pitch, the array's
        // distance from the sensor by similar triangles with the last element's aperture, then per
        // pinhole its chief ray from the superpixel centre through the lens centre, cut at that plane
        const int W = lens.num_pinholes_w, H = lens.num_pinholes_h;
        const float filmDistance = lens.film_distance;
        const float aspectRatio = (float)camera.xres / (float)camera.yres;
        const float width = lens.film_diag / sqrtf((1.f + 1.f / (aspectRatio * aspectRatio)));
        const float sPixPitch = width / ((float)W);
        const float lastAperture = lensEl[lensEl.size() - 1];
        const float pinholeArrayDistance = sPixPitch * filmDistance / (lastAperture + sPixPitch);
        const float pinholePosition = -filmDistance + pinholeArrayDistance;
        lensPinholes.assign((size_t)W * H * 3, 0.f);
        for (int i = 0; i < W; ++i)
            for (int j = 0; j < H; ++j) {
                const float cx = (float)(-(i - W / 2.0 + .5) * sPixPitch);
                const float cy = (float)((j - H / 2.0 + .5) * sPixPitch);
                const float cz = -filmDistance;
                // Normalize(lensCenter - centerPos): v / Length() = v * (1 / sqrtf(|v|^2)) (geometry.h)
                const float vx = 0.f - cx, vy = 0.f - cy, vz = 0.f - cz;
                const float inv = 1.f / sqrtf(vx * vx + vy * vy + vz * vz);
                const float dx = vx * inv, dy = vy * inv, dz = vz * inv;
                const float tHit = pinholePosition / dz;
                float *o = &lensPinholes[3 * ((size_t)i * H + j)];
                o[0] = tHit * dx;
                o[1] = tHit * dy;
                o[2] = pinholePosition;
            }
        f->lens.pinholes = lensPinholes.data();
    }
}

}  // namespace pbrtamd
