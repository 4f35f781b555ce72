// mano_diag.h -- the product build carries no diagnostic or tuning switch.
//
// The kernel sources keep their measured alternatives behind MANO_* macros
// (DESIGN.md §4 cites each A/B): ablations that return wrong results
// (MANO_BS_ABLATE, MANO_H3_ABLATE, MANO_QUAD_ABLATE, MANO_SPAN_ABLATE, the
// packed-fp32 MANO_H3_NO_PACK=0), clock stamps that add device globals
// (MANO_BS_STAMP, MANO_PAIR_STAMP) and geometry / priority knobs.  Only the
// builds under tools/ may set them, and they must say so with
// -DMANO_DIAGNOSTIC_BUILD (tools' builds write libraries of their own names;
// __graft_entry__.build_library adds the define for them).  Every knob the
// sources read is listed here (tests/test_codegen.py checks the list against
// the sources), so a product build that sets any of them does not compile.
#pragma once

#if !defined(MANO_DIAGNOSTIC_BUILD)
#if  defined(MANO_BS_ABLATE) || defined(MANO_BS_ACC2) || defined(MANO_BS_ALIGN) || defined(MANO_BS_BLOCKS_PER_CU) ||   \
    defined(MANO_BS_DMA_PRIO) || defined(MANO_BS_NT_STORE) || defined(MANO_BS_REST_NT) || defined(MANO_BS_STAMP) || \
    defined(MANO_BLEND_STORE_POLICY) || defined(MANO_BLEND_COUNTED) ||           \
    defined(MANO_BS_STORE_PRIO) || defined(MANO_H3_ABLATE) || defined(MANO_H3_ALIGN) || defined(MANO_H3_ASM_MFMA) ||         \
    defined(MANO_H3_BLOCKS) || defined(MANO_H3_DMA_PRIO) || defined(MANO_H3_FULL_WAIT) ||          \
    defined(MANO_H3_NO_PACK) || defined(MANO_H3_NT_STORE) || defined(MANO_H3_RING) || defined(MANO_H3_SPLIT_ACC) || defined(MANO_H3_SCALAR_UNSCALE) ||    \
    defined(MANO_H3_SKIN_PAIR) || defined(MANO_H3_TPW) || defined(MANO_H3_WAVES) ||                \
    defined(MANO_PAIR_POLL_LIMIT) || defined(MANO_PAIR_ALIGN) || defined(MANO_PAIR_NT) || defined(MANO_PAIR_REVERSE) || defined(MANO_PAIR_INPLACE_FORWARD) || defined(MANO_PAIR_INPLACE_ORDER) || defined(MANO_PAIR_INPLACE_HOT) || defined(MANO_PAIR_SLEEP_CMP) || defined(MANO_PAIR_SLEEP_MEM) || \
    defined(MANO_PAIR_SLOTS) || defined(MANO_PAIR_STAMP) || defined(MANO_QUAD_ABLATE) ||           \
    defined(MANO_QUAD_GROUP_MAJOR) || defined(MANO_QUAD_MAX_GROUPS) || defined(MANO_QUAD_PAIR) ||  \
    defined(MANO_QUAD_PAIR_COMPUTE) || defined(MANO_QUAD_PAIR_PRIO) || defined(MANO_QUAD_P_EARLY) || \
    defined(MANO_QUAD_WAVES) || defined(MANO_SKIN_QUAD) || defined(MANO_SPAN_ABLATE) ||            \
    defined(MANO_SPAN_BLOCKS_PER_CU) || defined(MANO_SPAN_CHUNK) ||                                \
    defined(MANO_SPAN_H3_BLOCKS_PER_CU) || defined(MANO_SPAN_H3_PRIO) ||                           \
    defined(MANO_SPAN_H3_STRIDE) || defined(MANO_SPAN_NT_LOAD) || defined(MANO_SPAN_VERTS)
#error "a MANO_* diagnostic / tuning switch is set in a product build (tools/ builds add -DMANO_DIAGNOSTIC_BUILD)"
#endif
#endif
