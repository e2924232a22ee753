// Hardware probe: do gfx950 MFMAs whose destination partially overlaps a source --
// and the exact instruction sequence of the intermittently wrong Swin build (K=16 bf16 MFMAs) --
// give the same bits as the same products on disjoint registers?  Standalone program:
//   hipcc -O2 --offload-arch=gfx950 tools/probe_mfma_overlap.hip -o build/probe_mfma_overlap
//   build/probe_mfma_overlap [iters]  -> one line per variant: mismatching result words / words checked
// Each variant runs a test form and a reference form (every operand in its own registers, 32 wait
// states between dependent instructions) in the same lane on the same operands, 2048 workgroups x
// 8 waves x 32 iterations; "hammer" runs the same with waves 4-7 issuing back-to-back 32x32x16
// MFMAs beside them, so the test waves' MFMAs wait for the shared matrix pipe.  Each lane writes
// only its own counters; no buffer is indexed out of bounds.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <vector>

#define CHECK(x)                                                                      \
  do {                                                                                \
    hipError_t e_ = (x);                                                              \
    if (e_ != hipSuccess) {                                                           \
      printf("HIP error %s at line %d\n", hipGetErrorString(e_), __LINE__);           \
      exit(2);                                                                        \
    }                                                                                 \
  } while (0)

constexpr int NB = 2048, NT = 512, NW = 24, NV = 18;

#define PAD "s_nop 7\n s_nop 7\n s_nop 7\n s_nop 7\n"
// operand words -> v[64:87]: A16 v[64:65], B16 v[66:67], C v[68:71], A32 v[72:75], B32 v[76:79],
// A32b v[80:83], A32c v[84:87]
#define LOADIN                                                                                           \
  "v_mov_b32 v64, %[i0]\n v_mov_b32 v65, %[i1]\n v_mov_b32 v66, %[i2]\n v_mov_b32 v67, %[i3]\n"          \
  "v_mov_b32 v68, %[i4]\n v_mov_b32 v69, %[i5]\n v_mov_b32 v70, %[i6]\n v_mov_b32 v71, %[i7]\n"          \
  "v_mov_b32 v72, %[i8]\n v_mov_b32 v73, %[i9]\n v_mov_b32 v74, %[i10]\n v_mov_b32 v75, %[i11]\n"        \
  "v_mov_b32 v76, %[i12]\n v_mov_b32 v77, %[i13]\n v_mov_b32 v78, %[i14]\n v_mov_b32 v79, %[i15]\n"      \
  "v_mov_b32 v80, %[i16]\n v_mov_b32 v81, %[i17]\n v_mov_b32 v82, %[i18]\n v_mov_b32 v83, %[i19]\n"      \
  "v_mov_b32 v84, %[i20]\n v_mov_b32 v85, %[i21]\n v_mov_b32 v86, %[i22]\n v_mov_b32 v87, %[i23]\n" PAD
#define IN_OPS                                                                                              \
  [i0] "v"(w[0]), [i1] "v"(w[1]), [i2] "v"(w[2]), [i3] "v"(w[3]), [i4] "v"(w[4]), [i5] "v"(w[5]),          \
      [i6] "v"(w[6]), [i7] "v"(w[7]), [i8] "v"(w[8]), [i9] "v"(w[9]), [i10] "v"(w[10]), [i11] "v"(w[11]),  \
      [i12] "v"(w[12]), [i13] "v"(w[13]), [i14] "v"(w[14]), [i15] "v"(w[15]), [i16] "v"(w[16]),            \
      [i17] "v"(w[17]), [i18] "v"(w[18]), [i19] "v"(w[19]), [i20] "v"(w[20]), [i21] "v"(w[21]),            \
      [i22] "v"(w[22]), [i23] "v"(w[23]), [lds] "v"(lds)
#define OUT_OPS                                                                                              \
  [o0] "=&v"(o[0]), [o1] "=&v"(o[1]), [o2] "=&v"(o[2]), [o3] "=&v"(o[3]), [o4] "=&v"(o[4]),                  \
      [o5] "=&v"(o[5]), [o6] "=&v"(o[6]), [o7] "=&v"(o[7]), [o8] "=&v"(o[8]), [o9] "=&v"(o[9]),              \
      [o10] "=&v"(o[10]), [o11] "=&v"(o[11]), [o12] "=&v"(o[12]), [o13] "=&v"(o[13]), [o14] "=&v"(o[14]),    \
      [o15] "=&v"(o[15])
// results: v[128:143] -> o[0:16]
#define STORE_R                                                                                            \
  PAD "v_mov_b32 %[o0], v128\n v_mov_b32 %[o1], v129\n v_mov_b32 %[o2], v130\n v_mov_b32 %[o3], v131\n"     \
      "v_mov_b32 %[o4], v132\n v_mov_b32 %[o5], v133\n v_mov_b32 %[o6], v134\n v_mov_b32 %[o7], v135\n"     \
      "v_mov_b32 %[o8], v136\n v_mov_b32 %[o9], v137\n v_mov_b32 %[o10], v138\n v_mov_b32 %[o11], v139\n"   \
      "v_mov_b32 %[o12], v140\n v_mov_b32 %[o13], v141\n v_mov_b32 %[o14], v142\n v_mov_b32 %[o15], v143\n"
#define ZERO_R                                                                                               \
  "v_mov_b32 v128, 0\n v_mov_b32 v129, 0\n v_mov_b32 v130, 0\n v_mov_b32 v131, 0\n v_mov_b32 v132, 0\n"      \
  "v_mov_b32 v133, 0\n v_mov_b32 v134, 0\n v_mov_b32 v135, 0\n v_mov_b32 v136, 0\n v_mov_b32 v137, 0\n"      \
  "v_mov_b32 v138, 0\n v_mov_b32 v139, 0\n v_mov_b32 v140, 0\n v_mov_b32 v141, 0\n v_mov_b32 v142, 0\n"      \
  "v_mov_b32 v143, 0\n"
#define CP4(d, s) "v_mov_b32 v" #d ", v" #s "\n"
#define RES(d0, s0) "v_mov_b32 v" #d0 ", v" #s0 "\n"
#define CLOB                                                                                                   \
  "v64", "v65", "v66", "v67", "v68", "v69", "v70", "v71", "v72", "v73", "v74", "v75", "v76", "v77", "v78", "v79", \
      "v80", "v81", "v82", "v83", "v84", "v85", "v86", "v87", "v88", "v89", "v90", "v91", "v92", "v93", "v94",    \
      "v95", "v96", "v97", "v98", "v99", "v100", "v101", "v102", "v103", "v104", "v105", "v106", "v107", "v108", \
      "v109", "v110", "v111", "v112", "v113", "v114", "v115", "v116", "v117", "v118", "v119", "v120", "v121",    \
      "v122", "v123", "v124", "v125", "v126", "v127", "v128", "v129", "v130", "v131", "v132", "v133", "v134",    \
      "v135", "v136", "v137", "v138", "v139", "v140", "v141", "v142", "v143", "memory"

#define RUN(BODY) asm volatile(LOADIN ZERO_R BODY STORE_R : OUT_OPS : IN_OPS : CLOB)

// one 16x16 MFMA's result in v[96:99] copied to v[128:131]
#define TO_R "v_mov_b32 v128, v96\n v_mov_b32 v129, v97\n v_mov_b32 v130, v98\n v_mov_b32 v131, v99\n"

template <int V, bool REF>
__device__ __forceinline__ void body(const uint32_t (&w)[NW], float (&o)[16], uint32_t lds) {
  // -------- single MFMAs: the reference puts dst in v[96:99], operands where LOADIN left them
  if constexpr (V <= 4) {      // K=16
    if constexpr (REF) {
      RUN("v_mfma_f32_16x16x16_bf16 v[96:99], v[64:65], v[66:67], v[68:71]\n" PAD TO_R);
    } else if constexpr (V == 0) {   // dst over srcA (upper half of dst)
      RUN("v_mov_b32 v98, v64\n v_mov_b32 v99, v65\n" PAD
          "v_mfma_f32_16x16x16_bf16 v[96:99], v[98:99], v[66:67], v[68:71]\n" PAD TO_R);
    } else if constexpr (V == 1) {   // dst over srcA (lower half)
      RUN("v_mov_b32 v96, v64\n v_mov_b32 v97, v65\n" PAD
          "v_mfma_f32_16x16x16_bf16 v[96:99], v[96:97], v[66:67], v[68:71]\n" PAD TO_R);
    } else if constexpr (V == 2) {   // dst over srcB
      RUN("v_mov_b32 v98, v66\n v_mov_b32 v99, v67\n" PAD
          "v_mfma_f32_16x16x16_bf16 v[96:99], v[64:65], v[98:99], v[68:71]\n" PAD TO_R);
    } else if constexpr (V == 3) {   // dst over srcC, shifted up
      RUN("v_mov_b32 v98, v68\n v_mov_b32 v99, v69\n v_mov_b32 v100, v70\n v_mov_b32 v101, v71\n" PAD
          "v_mfma_f32_16x16x16_bf16 v[96:99], v[64:65], v[66:67], v[98:101]\n" PAD TO_R);
    } else {                         // dst over srcC, shifted down
      RUN("v_mov_b32 v94, v68\n v_mov_b32 v95, v69\n v_mov_b32 v96, v70\n v_mov_b32 v97, v71\n" PAD
          "v_mfma_f32_16x16x16_bf16 v[96:99], v[64:65], v[66:67], v[94:97]\n" PAD TO_R);
    }
  } else if constexpr (V <= 9) {   // K=32
    if constexpr (REF) {
      RUN("v_mfma_f32_16x16x32_bf16 v[96:99], v[72:75], v[76:79], v[68:71]\n" PAD TO_R);
    } else if constexpr (V == 5) {   // dst over srcA
      RUN("v_mov_b32 v98, v72\n v_mov_b32 v99, v73\n v_mov_b32 v100, v74\n v_mov_b32 v101, v75\n" PAD
          "v_mfma_f32_16x16x32_bf16 v[96:99], v[98:101], v[76:79], v[68:71]\n" PAD TO_R);
    } else if constexpr (V == 6) {   // dst over srcB, shifted up
      RUN("v_mov_b32 v98, v76\n v_mov_b32 v99, v77\n v_mov_b32 v100, v78\n v_mov_b32 v101, v79\n" PAD
          "v_mfma_f32_16x16x32_bf16 v[96:99], v[72:75], v[98:101], v[68:71]\n" PAD TO_R);
    } else if constexpr (V == 7) {   // dst over srcB, shifted down
      RUN("v_mov_b32 v94, v76\n v_mov_b32 v95, v77\n v_mov_b32 v96, v78\n v_mov_b32 v97, v79\n" PAD
          "v_mfma_f32_16x16x32_bf16 v[96:99], v[72:75], v[94:97], v[68:71]\n" PAD TO_R);
    } else if constexpr (V == 8) {   // dst over srcC, shifted up
      RUN("v_mov_b32 v98, v68\n v_mov_b32 v99, v69\n v_mov_b32 v100, v70\n v_mov_b32 v101, v71\n" PAD
          "v_mfma_f32_16x16x32_bf16 v[96:99], v[72:75], v[76:79], v[98:101]\n" PAD TO_R);
    } else {                         // dst over srcC, shifted down
      RUN("v_mov_b32 v94, v68\n v_mov_b32 v95, v69\n v_mov_b32 v96, v70\n v_mov_b32 v97, v71\n" PAD
          "v_mfma_f32_16x16x32_bf16 v[96:99], v[72:75], v[76:79], v[94:97]\n" PAD TO_R);
    }
  } else if constexpr (V == 10 || V == 11) {
    // the sequence of the wrong Swin build (swin_window.hip at ffe1710, instance <true,true>),
    // registers renumbered 12->80, 24->84, 28->72(A32), 134->76(B32), instruction gaps kept:
    //   P1 = A32b.B32 (16x16x32, C=0) -> v[78:81] ... P2 = A32c.B32 -> v[82:85] (here: v[108:111])
    //   M1 = P1 + A16a.B16 -> v[78:81]   (K=16, srcA v[74:75])
    //   M2 = P2 + A16b.B16 -> v[74:77]   (K=16, dst over M1's srcA and its own srcA v[76:77])
    //   M3 = A32.B32 (C=0) -> v[82:85]  (16x16x32, dst over M2's srcC)
    // V 10: as issued; V 11: the same with the two K=16 products on the 16x16x32 form (B16 and
    // the A16 halves zero-extended to K=32: identical sums)
    if constexpr (REF && V == 11) {
      RUN("v_mov_b32 v88, v64\n v_mov_b32 v89, v65\n v_mov_b32 v90, 0\n v_mov_b32 v91, 0\n"
          "v_mov_b32 v92, v68\n v_mov_b32 v93, v69\n v_mov_b32 v94, 0\n v_mov_b32 v95, 0\n"
          "v_mov_b32 v96, v66\n v_mov_b32 v97, v67\n v_mov_b32 v98, 0\n v_mov_b32 v99, 0\n" PAD
          "v_mfma_f32_16x16x32_bf16 v[100:103], v[80:83], v[76:79], 0\n" PAD
          "v_mfma_f32_16x16x32_bf16 v[104:107], v[84:87], v[76:79], 0\n" PAD
          "v_mfma_f32_16x16x32_bf16 v[128:131], v[88:91], v[96:99], v[100:103]\n" PAD
          "v_mfma_f32_16x16x32_bf16 v[132:135], v[92:95], v[96:99], v[104:107]\n" PAD
          "v_mfma_f32_16x16x32_bf16 v[136:139], v[72:75], v[76:79], 0\n" PAD
          "v_mov_b32 v140, v130\n v_mov_b32 v141, v131\n v_mov_b32 v142, v134\n v_mov_b32 v143, v135\n");
    } else if constexpr (REF) {
      RUN("v_mfma_f32_16x16x32_bf16 v[100:103], v[80:83], v[76:79], 0\n" PAD
          "v_mfma_f32_16x16x32_bf16 v[104:107], v[84:87], v[76:79], 0\n" PAD
          "v_mfma_f32_16x16x16_bf16 v[128:131], v[64:65], v[66:67], v[100:103]\n" PAD
          "v_mfma_f32_16x16x16_bf16 v[132:135], v[68:69], v[66:67], v[104:107]\n" PAD
          "v_mfma_f32_16x16x32_bf16 v[136:139], v[72:75], v[76:79], 0\n" PAD
          "v_mov_b32 v140, v130\n v_mov_b32 v141, v131\n v_mov_b32 v142, v134\n v_mov_b32 v143, v135\n");
    } else if constexpr (V == 10) {
      RUN(// stage: A16a -> v[74:75] (=w0,w1), A16b -> v[76:77] (=w4,w5), B16 -> v[66:67] stays,
          // A32b -> v[112:115], A32c -> v[116:119], A32 -> v[120:123], B32 -> v[124:127]
          "v_mov_b32 v112, v80\n v_mov_b32 v113, v81\n v_mov_b32 v114, v82\n v_mov_b32 v115, v83\n"
          "v_mov_b32 v116, v84\n v_mov_b32 v117, v85\n v_mov_b32 v118, v86\n v_mov_b32 v119, v87\n"
          "v_mov_b32 v120, v72\n v_mov_b32 v121, v73\n v_mov_b32 v122, v74\n v_mov_b32 v123, v75\n"
          "v_mov_b32 v124, v76\n v_mov_b32 v125, v77\n v_mov_b32 v126, v78\n v_mov_b32 v127, v79\n" PAD
          "v_mov_b32 v74, v64\n v_mov_b32 v75, v65\n v_mov_b32 v76, v68\n v_mov_b32 v77, v69\n" PAD
          "v_mfma_f32_16x16x32_bf16 v[78:81], v[112:115], v[124:127], 0\n"
          "s_nop 0\n s_nop 0\n s_nop 0\n"
          "v_mfma_f32_16x16x32_bf16 v[82:85], v[116:119], v[124:127], 0\n"
          "s_nop 0\n s_nop 0\n s_nop 0\n s_nop 0\n"
          "v_mfma_f32_16x16x16_bf16 v[78:81], v[74:75], v[66:67], v[78:81]\n"
          "s_nop 0\n"
          "v_mfma_f32_16x16x16_bf16 v[74:77], v[76:77], v[66:67], v[82:85]\n"
          "v_mfma_f32_16x16x32_bf16 v[82:85], v[120:123], v[124:127], 0\n"
          "s_nop 4\n"
          "v_mov_b32 v140, v80\n v_mov_b32 v141, v81\n"
          "s_nop 0\n"
          "v_mov_b32 v142, v76\n v_mov_b32 v143, v77\n" PAD
          "v_mov_b32 v128, v78\n v_mov_b32 v129, v79\n v_mov_b32 v130, v80\n v_mov_b32 v131, v81\n"
          "v_mov_b32 v132, v74\n v_mov_b32 v133, v75\n v_mov_b32 v134, v76\n v_mov_b32 v135, v77\n"
          "v_mov_b32 v136, v82\n v_mov_b32 v137, v83\n v_mov_b32 v138, v84\n v_mov_b32 v139, v85\n");
    } else {
      RUN("v_mov_b32 v112, v80\n v_mov_b32 v113, v81\n v_mov_b32 v114, v82\n v_mov_b32 v115, v83\n"
          "v_mov_b32 v116, v84\n v_mov_b32 v117, v85\n v_mov_b32 v118, v86\n v_mov_b32 v119, v87\n"
          "v_mov_b32 v120, v72\n v_mov_b32 v121, v73\n v_mov_b32 v122, v74\n v_mov_b32 v123, v75\n"
          "v_mov_b32 v124, v76\n v_mov_b32 v125, v77\n v_mov_b32 v126, v78\n v_mov_b32 v127, v79\n" PAD
          // K=32 operands of the two K=16 products: A = [A16, 0, 0], B = [B16, 0, 0] (k 0..3 of
          // each lane group carry the K=16 product, k 4..7 contribute 0)
          "v_mov_b32 v88, v64\n v_mov_b32 v89, v65\n v_mov_b32 v90, 0\n v_mov_b32 v91, 0\n"
          "v_mov_b32 v92, v68\n v_mov_b32 v93, v69\n v_mov_b32 v94, 0\n v_mov_b32 v95, 0\n"
          "v_mov_b32 v96, v66\n v_mov_b32 v97, v67\n v_mov_b32 v98, 0\n v_mov_b32 v99, 0\n" PAD
          "v_mfma_f32_16x16x32_bf16 v[78:81], v[112:115], v[124:127], 0\n"
          "s_nop 0\n s_nop 0\n s_nop 0\n"
          "v_mfma_f32_16x16x32_bf16 v[82:85], v[116:119], v[124:127], 0\n"
          "s_nop 0\n s_nop 0\n s_nop 0\n s_nop 0\n"
          "v_mfma_f32_16x16x32_bf16 v[78:81], v[88:91], v[96:99], v[78:81]\n"
          "s_nop 0\n"
          "v_mfma_f32_16x16x32_bf16 v[90:93], v[92:95], v[96:99], v[82:85]\n"
          "v_mfma_f32_16x16x32_bf16 v[82:85], v[120:123], v[124:127], 0\n"
          "s_nop 4\n"
          "v_mov_b32 v140, v80\n v_mov_b32 v141, v81\n"
          "s_nop 0\n"
          "v_mov_b32 v142, v92\n v_mov_b32 v143, v93\n" PAD
          "v_mov_b32 v128, v78\n v_mov_b32 v129, v79\n v_mov_b32 v130, v80\n v_mov_b32 v131, v81\n"
          "v_mov_b32 v132, v90\n v_mov_b32 v133, v91\n v_mov_b32 v134, v92\n v_mov_b32 v135, v93\n"
          "v_mov_b32 v136, v82\n v_mov_b32 v137, v83\n v_mov_b32 v138, v84\n v_mov_b32 v139, v85\n");
    }
  } else if constexpr (V >= 14) {
    // the wrong Swin build's pattern (ffe1710, swin_win5<true,true>): MFMA B reads as srcC the
    // result of MFMA A issued two instructions earlier (so B waits in the matrix pipe for A), and
    // an LDS load into those srcC registers is issued 5 wait states after B.  V 14 / 15: B is
    // K=16 / K=32; V 16 / 17: the same with A's result made ready first (padded), B then issues
    // with no pending dependency.  P = A32b.B32 (16x16x32, C=0); B = A16.B16 + P (or A32.B32 + P)
    if constexpr (REF) {
      if constexpr (V == 14 || V == 16)
        RUN("v_mfma_f32_16x16x32_bf16 v[100:103], v[80:83], v[76:79], 0\n" PAD
            "v_mfma_f32_16x16x16_bf16 v[96:99], v[64:65], v[66:67], v[100:103]\n" PAD TO_R);
      else
        RUN("v_mfma_f32_16x16x32_bf16 v[100:103], v[80:83], v[76:79], 0\n" PAD
            "v_mfma_f32_16x16x32_bf16 v[96:99], v[72:75], v[76:79], v[100:103]\n" PAD TO_R);
    } else if constexpr (V == 14) {
      RUN("v_mfma_f32_16x16x32_bf16 v[100:103], v[80:83], v[76:79], 0\n"
          "s_nop 0\n"
          "v_mfma_f32_16x16x16_bf16 v[96:99], v[64:65], v[66:67], v[100:103]\n"
          "s_nop 4\n"
          "ds_read_b128 v[100:103], %[lds]\n"
          "s_waitcnt lgkmcnt(0)\n" PAD TO_R);
    } else if constexpr (V == 15) {
      RUN("v_mfma_f32_16x16x32_bf16 v[100:103], v[80:83], v[76:79], 0\n"
          "s_nop 0\n"
          "v_mfma_f32_16x16x32_bf16 v[96:99], v[72:75], v[76:79], v[100:103]\n"
          "s_nop 4\n"
          "ds_read_b128 v[100:103], %[lds]\n"
          "s_waitcnt lgkmcnt(0)\n" PAD TO_R);
    } else if constexpr (V == 16) {
      RUN("v_mfma_f32_16x16x32_bf16 v[100:103], v[80:83], v[76:79], 0\n" PAD
          "v_mfma_f32_16x16x16_bf16 v[96:99], v[64:65], v[66:67], v[100:103]\n"
          "s_nop 4\n"
          "ds_read_b128 v[100:103], %[lds]\n"
          "s_waitcnt lgkmcnt(0)\n" PAD TO_R);
    } else {
      RUN("v_mfma_f32_16x16x32_bf16 v[100:103], v[80:83], v[76:79], 0\n" PAD
          "v_mfma_f32_16x16x32_bf16 v[96:99], v[72:75], v[76:79], v[100:103]\n"
          "s_nop 4\n"
          "ds_read_b128 v[100:103], %[lds]\n"
          "s_waitcnt lgkmcnt(0)\n" PAD TO_R);
    }
  } else {
    // an LDS load landing in the srcC registers of a just-issued MFMA, 5 wait states later (the
    // padding hipcc gave the wrong Swin build): V 12 K=16, V 13 K=32.  The LDS words are 1e9f.
    if constexpr (REF) {
      if constexpr (V == 12) RUN("v_mfma_f32_16x16x16_bf16 v[96:99], v[64:65], v[66:67], v[68:71]\n" PAD TO_R);
      else RUN("v_mfma_f32_16x16x32_bf16 v[96:99], v[72:75], v[76:79], v[68:71]\n" PAD TO_R);
    } else if constexpr (V == 12) {
      RUN("v_mov_b32 v100, v68\n v_mov_b32 v101, v69\n v_mov_b32 v102, v70\n v_mov_b32 v103, v71\n" PAD
          "v_mfma_f32_16x16x16_bf16 v[96:99], v[64:65], v[66:67], v[100:103]\n"
          "s_nop 4\n"
          "ds_read_b128 v[100:103], %[lds]\n"
          "s_waitcnt lgkmcnt(0)\n" PAD TO_R);
    } else {
      RUN("v_mov_b32 v100, v68\n v_mov_b32 v101, v69\n v_mov_b32 v102, v70\n v_mov_b32 v103, v71\n" PAD
          "v_mfma_f32_16x16x32_bf16 v[96:99], v[72:75], v[76:79], v[100:103]\n"
          "s_nop 4\n"
          "ds_read_b128 v[100:103], %[lds]\n"
          "s_waitcnt lgkmcnt(0)\n" PAD TO_R);
    }
  }
}

typedef __attribute__((__vector_size__(8 * sizeof(__bf16)))) __bf16 bf16x8;
typedef __attribute__((__vector_size__(16 * sizeof(float)))) float f32x16;

template <int V>
__global__ __launch_bounds__(NT) void probe(const uint32_t* __restrict__ in, unsigned long long* __restrict__ bad,
                                            int hammer, int iters) {
  __shared__ float lds[NT * 4];
  for (int k = 0; k < 4; ++k) lds[threadIdx.x * 4 + k] = 1e9f;
  __syncthreads();
  const int wave = threadIdx.x >> 6;
  if (hammer && wave >= 4) {
    // partner waves: back-to-back independent 32x32x16 MFMAs on the same SIMDs
    bf16x8 a, b;
    for (int k = 0; k < 8; ++k) { a[k] = (__bf16)(0.001f * (threadIdx.x + k)); b[k] = (__bf16)(0.002f * k); }
    f32x16 acc[4] = {};
    for (int it = 0; it < iters * 6; ++it)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc[j], 0, 0, 0);
    float s = 0.f;
    for (int j = 0; j < 4; ++j) s += acc[j][0];
    if (s == 12345.678f) bad[NV * 2] = 1;      // keeps the chain live; never true for these inputs
    return;
  }
  const int64_t gid = (int64_t)blockIdx.x * NT + threadIdx.x;
  const uint32_t lds_addr = (uint32_t)(uintptr_t)&lds[threadIdx.x * 4];
  unsigned long long nb = 0;
  for (int it = 0; it < iters; ++it) {
    uint32_t w[NW];
    const uint32_t* src = in + (((gid * 7 + it * 131) & 65535) * NW);
    for (int k = 0; k < NW; ++k) w[k] = src[k];
    float t[16], r[16];
    body<V, false>(w, t, lds_addr);
    body<V, true>(w, r, lds_addr);
    for (int k = 0; k < 16; ++k) nb += __float_as_uint(t[k]) != __float_as_uint(r[k]);
  }
  if (nb) atomicAdd(bad + V, nb);
  atomicAdd(bad + NV + V, 1ull);     // lanes checked
}

template <int V>
void launch(const uint32_t* din, unsigned long long* dbad, int hammer, int iters) {
  hipLaunchKernelGGL(probe<V>, dim3(NB), dim3(NT), 0, 0, din, dbad, hammer, iters);
  if constexpr (V + 1 < NV) launch<V + 1>(din, dbad, hammer, iters);
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 32;   // iterations per wave (the test runs 4)
  if (iters < 1 || iters > 1024) { printf("bad iteration count\n"); return 2; }
  std::vector<uint32_t> h(65536 * NW);
  uint64_t s = 88172645463325252ull;
  for (size_t e = 0; e < h.size(); ++e) {
    s ^= s << 13; s ^= s >> 7; s ^= s << 17;
    const uint32_t r = (uint32_t)s;
    const int k = (int)(e % NW);
    // every word: two bf16 in +-[0.5, 2) (the accumulator words C are read as f32: still finite)
    const uint32_t lo = (0x3f00u + (r & 0xffu)) | ((r >> 8) & 1u) << 15;
    const uint32_t hi = (0x3f00u + ((r >> 9) & 0xffu)) | ((r >> 17) & 1u) << 15;
    h[e] = lo | (hi << 16);
  }
  uint32_t* din;
  unsigned long long* dbad;
  CHECK(hipMalloc(&din, h.size() * 4));
  CHECK(hipMemcpy(din, h.data(), h.size() * 4, hipMemcpyHostToDevice));
  CHECK(hipMalloc(&dbad, (2 * NV + 1) * 8));
  const char* names[NV] = {"k16 dst/srcA hi", "k16 dst/srcA lo", "k16 dst/srcB", "k16 dst/srcC up",
                           "k16 dst/srcC down", "k32 dst/srcA", "k32 dst/srcB up", "k32 dst/srcB down",
                           "k32 dst/srcC up", "k32 dst/srcC down", "swin K=16 sequence",
                           "swin sequence on K=32", "k16 LDS->srcC after 5 ws", "k32 LDS->srcC after 5 ws",
                           "k16 chained srcC + LDS", "k32 chained srcC + LDS", "k16 ready srcC + LDS",
                           "k32 ready srcC + LDS"};
  for (int hammer = 0; hammer < 2; ++hammer) {
    CHECK(hipMemset(dbad, 0, (2 * NV + 1) * 8));
    launch<0>(din, dbad, hammer, iters);
    CHECK(hipDeviceSynchronize());
    unsigned long long hb[2 * NV + 1];
    CHECK(hipMemcpy(hb, dbad, sizeof(hb), hipMemcpyDeviceToHost));
    for (int v = 0; v < NV; ++v)
      printf("%s %-26s mismatching words %llu of %llu\n", hammer ? "hammer" : "plain ", names[v], hb[v],
             hb[NV + v] * iters * 16);
  }
  return 0;
}
