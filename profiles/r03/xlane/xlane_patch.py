"""Insert a compiler memory barrier at every cross-lane LDS hand-over of the phase kernels
(pairing <-> natural layouts): entry of load_pair / load_cat_gl, end of squash_write's stores,
before each pairing-layout read of d loss / d a_d."""
import re, sys
root = sys.argv[1]
mlp = open(root + "/spp-rl_amd/csrc/mlp.h").read()
if "SPP_XLANE_SYNC" not in mlp:
    mlp = mlp.replace("namespace spp {", "namespace spp {\n#ifndef SPP_XLANE_SYNC\n#define SPP_XLANE_SYNC() asm volatile(\"\" ::: \"memory\")\n#endif\n", 1)
    open(root + "/spp-rl_amd/csrc/mlp.h", "w").write(mlp)
s = open(root + "/spp-rl_amd/csrc/sac.hip").read()
n0 = s.count("SPP_XLANE_SYNC")
s = s.replace("__device__ __forceinline__ void load_pair(f32x16 (&t)[C::NB_PAIR], const float* lds) {\n",
              "__device__ __forceinline__ void load_pair(f32x16 (&t)[C::NB_PAIR], const float* lds) {\n  SPP_XLANE_SYNC();\n", 1)
s = re.sub(r"(__device__ __forceinline__ void load_cat_gl\([^{]*\{\n)", r"\1  SPP_XLANE_SYNC();\n", s, count=1)
s = s.replace("  const float tot = lp + __shfl_xor(lp, 32, 64);\n", "  SPP_XLANE_SYNC();\n  const float tot = lp + __shfl_xor(lp, 32, 64);\n", 1)
s = re.sub(r"\n(\s*)float g_ad = L\.pl\[j0 \* 32\];", r"\n\1SPP_XLANE_SYNC();\n\1float g_ad = L.pl[j0 * 32];", s)
open(root + "/spp-rl_amd/csrc/sac.hip", "w").write(s)
print("barriers:", s.count("SPP_XLANE_SYNC") - n0)
