// Batched Internet (RFC 1071) checksum for MI355X (gfx950, CDNA4).
//
// The reference computes compute_ones_comp (src/stack/util.rs:88-106) once per
// packet on whichever CPU thread handles it.  Here a batch of
// packets already resident in HBM is checksummed by one launch:
//
//   * a packet is owned by a GROUP of G lanes (G = 4..64, a power of two, so a
//     64-lane wavefront serves 64/G packets at once); the group streams the
//     packet as 16-byte aligned chunks, lane l taking chunks l, l+G, ...,
//     U chunks in flight per lane (global_load_dwordx4, fully coalesced);
//   * bytes outside [start, start+len) in the first / last chunk are masked
//     to zero, so packets may start at any byte offset and the odd final
//     byte is the zero-padded word the reference adds as byte << 8;
//   * each dword is split by two v_dot4_u32_u8 into the sum of the bytes that
//     are the HIGH half of a big-endian word and the sum of the LOW halves
//     (which is which depends on the packet start's parity).  The reference's
//     u32 accumulator is exactly  seed + 256*high + low  (mod 2^32), so the
//     per-lane u32 partials are summed with wrap-around across the group
//     (shuffle butterfly) and folded end-around exactly like util.rs:101-103:
//     bit-exact for every length, including the reference's wrap past 128 KiB;
//   * one lane per group stores the u16 result (optionally ^ 0xffff).
//
// This is a bandwidth-bound integer reduction (~1 byte of HBM per 0.5 VALU
// op): no MFMA, no LDS staging needed for the data itself.  Roofline: HBM read
// bandwidth; algorithmic bytes per packet = len + 2.
#pragma once

// The device code, by kernel family (each part includes the one before it):
#include "rns_k_common.hpp"
#include "rns_k_rounds.hpp"
#include "rns_k_mixed.hpp"
#include "rns_k_chain.hpp"
#include "rns_k_stream.hpp"
#include "rns_k_rows.hpp"
