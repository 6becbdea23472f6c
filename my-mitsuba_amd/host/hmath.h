// Host-side math for the scene loader / kd-tree builder (Mitsuba-mirror side
// of the boundary).  Float32 like the reference's SINGLE_PRECISION build
// (build/config-linux-gcc.py:7); matrix inverses are done in double.
#pragma once
#include <cmath>
#include <cstdint>
#include <algorithm>
#include <stdexcept>
#include <string>

namespace mtsh {

struct V3 {
    float x = 0, y = 0, z = 0;
    V3() = default;
    V3(float a, float b, float c) : x(a), y(b), z(c) {}
    explicit V3(float a) : x(a), y(a), z(a) {}
    float &operator[](int i) { return (&x)[i]; }
    float operator[](int i) const { return (&x)[i]; }
    V3 operator+(const V3 &o) const { return {x + o.x, y + o.y, z + o.z}; }
    V3 operator-(const V3 &o) const { return {x - o.x, y - o.y, z - o.z}; }
    V3 operator-() const { return {-x, -y, -z}; }
    V3 operator*(float s) const { return {x * s, y * s, z * s}; }
    V3 operator/(float s) const { float r = 1.0f / s; return {x * r, y * r, z * r}; }
    V3 &operator+=(const V3 &o) { x += o.x; y += o.y; z += o.z; return *this; }
    V3 &operator-=(const V3 &o) { x -= o.x; y -= o.y; z -= o.z; return *this; }
    V3 &operator*=(float s) { x *= s; y *= s; z *= s; return *this; }
    V3 &operator/=(float s) { float r = 1.0f / s; x *= r; y *= r; z *= r; return *this; }
    bool isZero() const { return x == 0 && y == 0 && z == 0; }
};
inline V3 operator*(float s, const V3 &v) { return v * s; }
inline float dot(const V3 &a, const V3 &b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
inline V3 cross(const V3 &a, const V3 &b) {
    return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
}
inline float length(const V3 &a) { return std::sqrt(dot(a, a)); }
inline V3 normalize(const V3 &a) { return a / length(a); }
inline V3 vmin(const V3 &a, const V3 &b) { return {std::min(a.x, b.x), std::min(a.y, b.y), std::min(a.z, b.z)}; }
inline V3 vmax(const V3 &a, const V3 &b) { return {std::max(a.x, b.x), std::max(a.y, b.y), std::max(a.z, b.z)}; }

// util.cpp coordinateSystem (reference src/libcore/util.cpp:590-600)
inline void coordinateSystem(const V3 &a, V3 &b, V3 &c) {
    if (std::abs(a.x) > std::abs(a.y)) {
        float invLen = 1.0f / std::sqrt(a.x * a.x + a.z * a.z);
        c = V3(a.z * invLen, 0.0f, -a.x * invLen);
    } else {
        float invLen = 1.0f / std::sqrt(a.y * a.y + a.z * a.z);
        c = V3(0.0f, a.z * invLen, -a.y * invLen);
    }
    b = cross(c, a);
}

struct AABB {
    V3 mn{INFINITY, INFINITY, INFINITY}, mx{-INFINITY, -INFINITY, -INFINITY};
    void expand(const V3 &p) { mn = vmin(mn, p); mx = vmax(mx, p); }
    void expand(const AABB &b) { mn = vmin(mn, b.mn); mx = vmax(mx, b.mx); }
    bool valid() const { return mx.x >= mn.x && mx.y >= mn.y && mx.z >= mn.z; }
    V3 extents() const { return mx - mn; }
    float surfaceArea() const {
        V3 d = extents();
        return 2.0f * (d.x * d.y + d.y * d.z + d.z * d.x);
    }
    void clip(const AABB &b) { mn = vmax(mn, b.mn); mx = vmin(mx, b.mx); }
};

// 4x4 affine/projective transform with cached inverse (include/mitsuba/core/transform.h)
struct Transform {
    float m[4][4], inv[4][4];
    Transform() {
        for (int i = 0; i < 4; i++)
            for (int j = 0; j < 4; j++) m[i][j] = inv[i][j] = (i == j) ? 1.0f : 0.0f;
    }
    static Transform fromMatrix(const double a[4][4]) {
        Transform t;
        double b[4][4];
        invert4(a, b);
        for (int i = 0; i < 4; i++)
            for (int j = 0; j < 4; j++) { t.m[i][j] = (float)a[i][j]; t.inv[i][j] = (float)b[i][j]; }
        return t;
    }
    static Transform fromMatrixF(const float a[4][4]) {
        double d[4][4];
        for (int i = 0; i < 4; i++)
            for (int j = 0; j < 4; j++) d[i][j] = a[i][j];
        return fromMatrix(d);
    }
    Transform inverse() const {
        Transform t;
        for (int i = 0; i < 4; i++)
            for (int j = 0; j < 4; j++) { t.m[i][j] = inv[i][j]; t.inv[i][j] = m[i][j]; }
        return t;
    }
    Transform operator*(const Transform &o) const {
        Transform r;
        for (int i = 0; i < 4; i++)
            for (int j = 0; j < 4; j++) {
                double s = 0, si = 0;
                for (int k = 0; k < 4; k++) { s += (double)m[i][k] * o.m[k][j]; si += (double)o.inv[i][k] * inv[k][j]; }
                r.m[i][j] = (float)s; r.inv[i][j] = (float)si;
            }
        return r;
    }
    V3 point(const V3 &p) const {
        float x = m[0][0] * p.x + m[0][1] * p.y + m[0][2] * p.z + m[0][3];
        float y = m[1][0] * p.x + m[1][1] * p.y + m[1][2] * p.z + m[1][3];
        float z = m[2][0] * p.x + m[2][1] * p.y + m[2][2] * p.z + m[2][3];
        float w = m[3][0] * p.x + m[3][1] * p.y + m[3][2] * p.z + m[3][3];
        if (w == 1.0f) return {x, y, z};
        return V3(x, y, z) / w;
    }
    V3 pointAffine(const V3 &p) const {
        return {m[0][0] * p.x + m[0][1] * p.y + m[0][2] * p.z + m[0][3],
                m[1][0] * p.x + m[1][1] * p.y + m[1][2] * p.z + m[1][3],
                m[2][0] * p.x + m[2][1] * p.y + m[2][2] * p.z + m[2][3]};
    }
    V3 vector(const V3 &v) const {
        return {m[0][0] * v.x + m[0][1] * v.y + m[0][2] * v.z,
                m[1][0] * v.x + m[1][1] * v.y + m[1][2] * v.z,
                m[2][0] * v.x + m[2][1] * v.y + m[2][2] * v.z};
    }
    // Normals transform with the inverse transpose (transform.h operator()(Normal))
    V3 normal(const V3 &n) const {
        return {inv[0][0] * n.x + inv[1][0] * n.y + inv[2][0] * n.z,
                inv[0][1] * n.x + inv[1][1] * n.y + inv[2][1] * n.z,
                inv[0][2] * n.x + inv[1][2] * n.y + inv[2][2] * n.z};
    }
    bool isIdentity() const {
        for (int i = 0; i < 4; i++)
            for (int j = 0; j < 4; j++)
                if (m[i][j] != ((i == j) ? 1.0f : 0.0f)) return false;
        return true;
    }

    static Transform translate(const V3 &v) {
        double a[4][4] = {{1, 0, 0, v.x}, {0, 1, 0, v.y}, {0, 0, 1, v.z}, {0, 0, 0, 1}};
        return fromMatrix(a);
    }
    static Transform scale(const V3 &v) {
        double a[4][4] = {{v.x, 0, 0, 0}, {0, v.y, 0, 0}, {0, 0, v.z, 0}, {0, 0, 0, 1}};
        return fromMatrix(a);
    }
    // transform.cpp Transform::rotate (Rodrigues, angle in degrees)
    static Transform rotate(const V3 &axis_, float angleDeg) {
        V3 axis = normalize(axis_);
        double a = angleDeg * M_PI / 180.0;
        double s = std::sin(a), c = std::cos(a);
        double x = axis.x, y = axis.y, z = axis.z;
        double r[4][4] = {
            {x * x + (1 - x * x) * c, x * y * (1 - c) - z * s, x * z * (1 - c) + y * s, 0},
            {x * y * (1 - c) + z * s, y * y + (1 - y * y) * c, y * z * (1 - c) - x * s, 0},
            {x * z * (1 - c) - y * s, y * z * (1 - c) + x * s, z * z + (1 - z * z) * c, 0},
            {0, 0, 0, 1}};
        return fromMatrix(r);
    }
    // transform.cpp:99-123
    static Transform perspective(float fov, float clipNear, float clipFar) {
        double recip = 1.0 / ((double)clipFar - clipNear);
        double cot = 1.0 / std::tan((fov / 2.0) * M_PI / 180.0);
        double a[4][4] = {{cot, 0, 0, 0},
                          {0, cot, 0, 0},
                          {0, 0, clipFar * recip, -(double)clipNear * clipFar * recip},
                          {0, 0, 1, 0}};
        return fromMatrix(a);
    }
    // transform.cpp:191-214
    static Transform lookAt(const V3 &p, const V3 &t, const V3 &up) {
        V3 dir = t - p;
        if (length(dir) == 0) throw std::runtime_error("lookAt(): 'origin' and 'target' coincide!");
        dir = normalize(dir);
        V3 left = cross(up, dir);
        if (length(left) == 0)
            throw std::runtime_error("lookAt(): the forward and upward direction must be linearly independent!");
        left = normalize(left);
        V3 newUp = cross(dir, left);
        double a[4][4] = {{left.x, newUp.x, dir.x, p.x},
                          {left.y, newUp.y, dir.y, p.y},
                          {left.z, newUp.z, dir.z, p.z},
                          {0, 0, 0, 1}};
        return fromMatrix(a);
    }

    static void invert4(const double a[4][4], double out[4][4]) {
        double m[4][8];
        for (int i = 0; i < 4; i++)
            for (int j = 0; j < 8; j++) m[i][j] = j < 4 ? a[i][j] : (j - 4 == i ? 1.0 : 0.0);
        for (int c = 0; c < 4; c++) {
            int piv = c;
            for (int r = c + 1; r < 4; r++)
                if (std::abs(m[r][c]) > std::abs(m[piv][c])) piv = r;
            if (std::abs(m[piv][c]) < 1e-300) {
                for (int i = 0; i < 4; i++)
                    for (int j = 0; j < 4; j++) out[i][j] = 0;
                return;  // singular; caller validates
            }
            if (piv != c)
                for (int j = 0; j < 8; j++) std::swap(m[c][j], m[piv][j]);
            double d = m[c][c];
            for (int j = 0; j < 8; j++) m[c][j] /= d;
            for (int r = 0; r < 4; r++)
                if (r != c) {
                    double f = m[r][c];
                    if (f != 0)
                        for (int j = 0; j < 8; j++) m[r][j] -= f * m[c][j];
                }
        }
        for (int i = 0; i < 4; i++)
            for (int j = 0; j < 4; j++) out[i][j] = m[i][j + 4];
    }
};

}  // namespace mtsh
