"""Timing-only diagnostic variants of the 32-pixel splats, applied to a tree COPY (ab/<name>/), never to the product:
   python tools/diag_patch.py <copy root> <variant>...
variants:
  nomfma    mfma32h / mfma32b return their accumulator untouched (no MFMA issued; operands still formed)
  fwdnoepi  k_fwd32_l1 stops after the four waves' sums (no split-tile fan-in, L1 epilogue, fragments or view loss;
            nothing stored)
  fwdnouf   k_fwd32_l1 without the upstream fragments for the backward
  fwdnol1   k_fwd32_l1 without the per-pixel outputs and L1 terms
  bwdrega   k_bwd32 takes its A fragments from two registers (no LDS reads of the upstream fragments)
Outputs are garbage; only the kernels' times (tools/splat_probe.py) mean anything."""
import sys

root, variants = sys.argv[1], sys.argv[2:]
path = root + "/3dgaussian_amd/csrc/gr_hip.hip"
src = open(path).read()


def sub(old, new, count=1):
    global src
    assert src.count(old) == count, (old, src.count(old))
    src = src.replace(old, new)


for v in variants:
    if v == "nomfma":
        sub("  return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8_t, a), __builtin_bit_cast(f16x8_t, b), c, 0, 0, 0);",
            '  asm volatile("" : "+v"(c) : "v"(a), "v"(b));\n  return c;')
        sub("  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);\n}\n// offset of kslot",
            '  asm volatile("" : "+v"(c) : "v"(a), "v"(b));\n  return c;\n}\n// offset of kslot')
    elif v == "fwdnoepi":
        anchor = "        acc[q][2 * round + cc] = ((b[0] + b[2 * T32 * F32_LD]) + b[4 * T32 * F32_LD]) + b[6 * T32 * F32_LD];\n      }\n    }\n  }\n  const int nch = tile_chunks(ranges[2 * tile], ch) + tile_chunks(ranges[2 * tile + 1], ch);\n  if (nch > 1) {\n    // a tile split over several items: each leaves its partial sums (write-through)"
        sub(anchor, anchor.split("  const int nch")[0] + "  asm volatile(\"\" :: \"v\"(acc[0][0]), \"v\"(acc[1][1]), \"v\"(acc[2][2]), \"v\"(acc[3][3]));\n  return;\n" + "  const int nch" + anchor.split("  const int nch")[1])
    elif v == "bwdrega":  # k_bwd32's upstream fragments from two register-resident constants instead of LDS
        sub("      auto contract = [&](int side, int c, const s16x8 (&B)[2][2]) {",
            "      s16x8 fA0, fA1;\n      for (int j = 0; j < 8; ++j) { fA0[j] = (short)(lane + j); fA1[j] = (short)(lane - j); }\n      auto contract = [&](int side, int c, const s16x8 (&B)[2][2]) {")
        # (each use made opaque by an empty asm, so the compiler cannot fold the now identical contractions together)
        sub("        for (int s = 0; s < 2; ++s) d = mfma32h(as_frag(A0[(s * 2 + 1) * 64 + lane]), B[s][0], d);",
            "        for (int s = 0; s < 2; ++s) { s16x8 a1 = fA1; asm volatile(\"\" : \"+v\"(a1)); d = mfma32h(a1, B[s][0], d); }")
        sub("          const s16x8 a0 = as_frag(A0[(s * 2) * 64 + lane]);", "          s16x8 a0 = fA0; asm volatile(\"\" : \"+v\"(a0)); (void)A0;")
    elif v == "fwdnouf":  # k_fwd32_l1 without the backward's upstream fragments
        sub("  if (nch > 0) {  // an empty tile has no backward work item: no fragments", "  if (nch < 0) {")
    elif v == "fwdnol1":  # k_fwd32_l1 without the per-pixel outputs and L1 terms (u = the pixel sums)
        sub("""      write_pixel(v, p, a5, out_rgb, out_alpha, nullptr, nullptr, nullptr);
      float lr = 0.f, ls = 0.f;
      pixel_upstream(v, p, make_float4(acc[q][0], acc[q][1], acc[q][2], acc[q][3]), 0.0f, nullptr, nullptr, nullptr, l1,
                     u[q], lr, ls);""", """      (void)a5;
      float lr = acc[q][0], ls = 0.f;
      for (int c = 0; c < 4; ++c) u[q][c] = acc[q][c];""")
    else:
        raise SystemExit("unknown variant " + v)
open(path, "w").write(src)
print("patched", path, variants)
