"""Sum the VALU issue cost (cycles per wave64 instruction per SIMD, measured by tools/valu_microbench.hip on
MI355X) of the instructions between two line numbers of a gfx950 assembly listing."""
import re, sys
TWO = {"v_fma_f32", "v_fmac_f32", "v_mul_f32", "v_add_f32", "v_sub_f32", "v_subrev_f32", "v_add_u32", "v_sub_u32",
       "v_subrev_u32", "v_xor_b32", "v_and_b32", "v_or_b32", "v_ashrrev_i32", "v_mov_b32", "v_lshlrev_b16",
       "v_not_b32", "v_lshrrev_b32"}
EIGHT = {"v_sqrt_f32", "v_rcp_f32", "v_pk_fma_f32", "v_pk_add_f32", "v_pk_mul_f32", "v_rsq_f32", "v_exp_f32", "v_log_f32", "v_sin_f32", "v_cos_f32"}
path, a, b = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
tot, n, per = 0, 0, {}
for line in open(path).read().splitlines()[a - 1:b]:
    m = re.match(r"\s+(v_[a-z0-9_]+)", line)
    if not m:
        continue
    op = re.sub(r"_e(32|64)$", "", m.group(1))
    c = 2 if op in TWO else 8 if op in EIGHT else 4
    tot += c; n += 1
    per[op] = per.get(op, 0) + c
print(f"{n} VALU instructions, {tot} issue cycles")
for k, v in sorted(per.items(), key=lambda x: -x[1]):
    print(f"  {k:24s} {v}")
