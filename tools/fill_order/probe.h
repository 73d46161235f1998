// The expression form of the reference's Random() (Utils/Math.cuh:231-234): a Vec3 built from three calls of
// one side-effecting draw function in a single constructor call, Vec3(f(s), f(s), f(s)).  C++ leaves the
// order of the three calls unspecified; whichever call runs first gets draw 1.  The probe records which draw
// lands in x, y and z for a compiler.
#pragma once
#ifndef PROBE_QUAL
#define PROBE_QUAL
#endif
struct Vec3p {
    float e[3];
    PROBE_QUAL Vec3p(float a, float b, float c) { e[0] = a; e[1] = b; e[2] = c; }
};
struct Draws {
    unsigned n;
};
PROBE_QUAL inline float draw(Draws* s) { return (float)(++s->n); }  // 1, 2, 3 in call order
PROBE_QUAL inline Vec3p random_vec(Draws* s) { return Vec3p(draw(s), draw(s), draw(s)); }
