// render_kernel_brute.cpp — the REFERENCE's own source/render_kernel.cpp, compiled
// unchanged with USE_BVH 0 (test infrastructure, container-only).
//
// render_kernel.h fixes `#define USE_BVH 1` (render_kernel.h:13), so INTERSECT_SCENE
// (render_kernel.cpp:504-511) always takes the octree walk in the reference's build.
// Including the header first (its include guard then makes the .cpp's own include a
// no-op) and redefining the macro before the .cpp text is compiled selects the
// brute-force intersect_scene loop (render_kernel.cpp:453-483) instead. No reference
// text is copied or edited; the Makefile links this object in place of
// render_kernel.o into ref_driver_brute, which renders the reference's USE_BVH 0 path.
#include "render_kernel.h"
#undef USE_BVH
#define USE_BVH 0
#include "source/render_kernel.cpp"
