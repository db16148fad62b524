#!/usr/bin/env python3
"""Dispatch-latency microbenchmarks for the assembly interpreter design (gfx950).
k_smem:  dependent chain of s_load_dword (pointer chase in a small table)  -> SMEM hit latency
k_jump:  chain of s_setpc_b64 through 64 stubs 64 B apart                 -> computed-jump latency
k_disp:  s_load_dwordx8 entry + s_waitcnt + s_setpc chain (the interpreter's dispatch)
Each kernel stores (s_memtime delta, iterations) per wave to out[wave]."""
import sys
L = ['.amdgcn_target "amdgcn-amd-amdhsa--gfx950"', '.amdhsa_code_object_version 5', '.text']
def kern(name, body):
    global L
    L += ['.globl %s' % name, '.p2align 8', '.type %s,@function' % name, '%s:' % name]
    # s[0:1] kernarg: out ptr (8), table ptr (8), iters (4)
    L += ['s_load_dwordx4 s[4:7], s[0:1], 0x0', 's_load_dword s10, s[0:1], 0x10', 's_waitcnt lgkmcnt(0)',
          's_memtime s[12:13]', 's_waitcnt lgkmcnt(0)']
    L += body
    L += ['s_memtime s[14:15]', 's_waitcnt lgkmcnt(0)',
          's_sub_u32 s14, s14, s12', 's_subb_u32 s15, s15, s13',
          'v_mov_b32 v2, s14', 'v_mov_b32 v3, s15',
          'v_mov_b32 v4, s2', 'v_lshlrev_b32 v4, 3, v4', 'v_mov_b32 v5, 0',
          'v_lshl_add_u64 v[4:5], v[4:5], 0, s[4:5]',
          'v_cmp_eq_u32 vcc, 0, v0', 's_and_b64 exec, exec, vcc',
          'global_store_dwordx2 v[4:5], v[2:3], off', 's_waitcnt vmcnt(0)', 's_endpgm']
# smem chase: table[i] = next offset (bytes)
kern('k_smem', ['s_mov_b32 s16, 0', '.Lsm:', 's_load_dword s16, s[6:7], s16', 's_waitcnt lgkmcnt(0)',
               's_sub_u32 s10, s10, 1', 's_cmp_lg_u32 s10, 0', 's_cbranch_scc1 .Lsm'])
# jump chain: 64 stubs, each 64 B; the last one loops back while iters remain
body = ['s_getpc_b64 s[20:21]', '.Ljb:', 's_add_u32 s20, s20, .Lstub0-.Ljb', 's_addc_u32 s21, s21, 0',
        's_mov_b64 s[22:23], s[20:21]', 's_setpc_b64 s[20:21]', '.p2align 6']
for i in range(64):
    body += ['.Lstub%d:' % i, 's_add_u32 s20, s20, 64', 's_addc_u32 s21, s21, 0']
    if i == 63:
        body += ['s_sub_u32 s10, s10, 1', 's_cmp_lg_u32 s10, 0', 's_cbranch_scc0 .Ljdone',
                 's_mov_b64 s[20:21], s[22:23]', 's_setpc_b64 s[20:21]']
    else:
        body += ['s_setpc_b64 s[20:21]']
    body += ['.p2align 6']
body += ['.Ljdone:']
kern('k_jump', body)
# dispatch chain: table of 32-B entries {handler(8), pad, next_off(4 @16)}, handlers = stubs
body = ['s_mov_b32 s24, 0', 's_load_dwordx8 s[32:39], s[6:7], s24', 's_waitcnt lgkmcnt(0)', 's_setpc_b64 s[32:33]',
        '.p2align 6']
for i in range(64):
    body += ['.Ldh%d:' % i, 's_mov_b32 s24, s36']
    if i == 63:
        body += ['s_sub_u32 s10, s10, 1', 's_cmp_lg_u32 s10, 0', 's_cbranch_scc0 .Lddone']
    body += ['s_load_dwordx8 s[32:39], s[6:7], s24', 's_waitcnt lgkmcnt(0)', 's_setpc_b64 s[32:33]', '.p2align 6']
body += ['.Lddone:']
kern('k_disp', body)
# helper kernel: write handler addresses of k_disp stubs into table (entry i -> .Ldh(i), next=(i+1)%64)
L += ['.globl k_init', '.p2align 8', '.type k_init,@function', 'k_init:',
      's_load_dwordx4 s[4:7], s[0:1], 0x0', 's_getpc_b64 s[8:9]', '.Likb:', 's_waitcnt lgkmcnt(0)']
for i in range(64):
    L += ['s_mov_b64 s[10:11], s[8:9]', 's_add_u32 s10, s10, .Ldh%d-.Likb' % i, 's_addc_u32 s11, s11, -1',
          'v_mov_b32 v2, s10', 'v_mov_b32 v3, s11', 'v_mov_b32 v1, %d' % (((i + 1) % 64) * 32),
          'v_mov_b32 v4, %d' % (i * 32), 'v_mov_b32 v5, 0', 'v_lshl_add_u64 v[4:5], v[4:5], 0, s[6:7]',
          'global_store_dwordx2 v[4:5], v[2:3], off', 'global_store_dword v[4:5], v1, off offset:16']
L += ['s_waitcnt vmcnt(0)', 's_endpgm']
L += ['.rodata']
for k in ('k_smem', 'k_jump', 'k_disp', 'k_init'):
    L += ['.p2align 6', '.amdhsa_kernel %s' % k, '.amdhsa_next_free_vgpr 8', '.amdhsa_next_free_sgpr 48',
          '.amdhsa_accum_offset 8', '.amdhsa_user_sgpr_count 2', '.amdhsa_user_sgpr_kernarg_segment_ptr 1',
          '.amdhsa_system_sgpr_workgroup_id_x 1', '.amdhsa_kernarg_size 24', '.end_amdhsa_kernel']
L += ['.text', '.amdgpu_metadata', '---', 'amdhsa.kernels:']
for k in ('k_smem', 'k_jump', 'k_disp', 'k_init'):
    L += ['  - .args:', '      - .offset: 0', '        .size: 24', '        .value_kind: by_value',
          '    .group_segment_fixed_size: 0', '    .kernarg_segment_align: 8', '    .kernarg_segment_size: 24',
          '    .max_flat_workgroup_size: 64', '    .name: %s' % k, '    .private_segment_fixed_size: 0',
          '    .sgpr_count: 48', '    .symbol: %s.kd' % k, '    .vgpr_count: 8', '    .wavefront_size: 64']
L += ['amdhsa.target: amdgcn-amd-amdhsa--gfx950', 'amdhsa.version:', '  - 1', '  - 2', '...', '.end_amdgpu_metadata']
open(sys.argv[1], 'w').write('\n'.join(L) + '\n')
