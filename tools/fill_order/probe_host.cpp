// Host build of the Random() fill-order probe (probe.h): prints the draw index in x, y, z.
#include <cstdio>
#include "probe.h"
int main() {
    Draws s{0};
    volatile Vec3p v = random_vec(&s);
    std::printf("x=%g y=%g z=%g -> %s\n", v.e[0], v.e[1], v.e[2],
                v.e[0] == 1.0f ? "left-to-right" : (v.e[2] == 1.0f ? "right-to-left" : "other"));
    return 0;
}
