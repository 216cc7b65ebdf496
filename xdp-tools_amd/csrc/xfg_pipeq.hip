// SPDX-License-Identifier: GPL-2.0
//
// xfg_pipeq.hip — the IPv4-key pipelined classify over the quotient index
// (kargs.qt; layout: xfg_layout.h).  Included by xfg_kernels.hip after
// xfg_pipeline.hip, whose parse (parse_bf), port probe and packing it uses.
//
// Why: the reference program's map lookup (CHECK_MAP,
// xdp-filter/xdpfilt_prog.h:56-64) is a random access per packet.  On
// gfx950 random requests cost on top of the frame stream (measured:
// tools/mb_pipe.hip, profiles/r03_mb_*): a prefilter word plus a 64-byte
// line for half the packets from the 8.9 MB canonical table took 1.16-1.19
// ms per 2^26 packets, one 32/64-byte bucket per packet from a <= 4 MB
// table 0.95.  The quotient index is that table: 2^bits buckets of 15
// entries, a bijective key hash so that a bucket's 15-bit remainders
// identify their keys exactly, and the one live direction's mask bit per
// entry -- so a lookup is ONE random 32-byte read, no prefilter hop.
//
// Used when exactly one IPv4 lookup direction can hit (flag census), every
// device carries the same flags, and the map is large (xfg_ctx.c
// fill_kargs).  Results are identical to xfg_pipe4_kernel's: a miss in a
// bucket that overflowed, and every shape the static parse does not cover,
// go to the deferred list and the canonical table (classify_staged).
//
// Per wave, iteration k works on three tiles of 64 packets:
//   R  tile k-1's buckets (LDS-DMA'd by L last iteration): match -> verdict
//   W  tile k-1's verdict stores, counters, stats, deferrals
//   S  tile k's windows (loaded two iterations ago) into the LDS rows
//   P  parse tile k, hash its key, plan its fallback (ports from LDS)
//   L  tile k's buckets, LDS-DMA'd into the rows (two lanes a bucket)
//   I  tile k+2's windows and lengths issued
// One wait per iteration, at its top: everything but the newest tile's
// CPP + 2 loads.
namespace {

template <uint32_t FEAT, int W, bool DENSE>
__global__ __launch_bounds__(PIPE_THREADS(W), (W) <= 64 ? 4 : 2) void xfg_pipeq_kernel(const xfg_kargs a)
{
	static_assert((FEAT & F_IPV4) != 0, "IPv4-key mode needs the IPv4 feature");
	constexpr int NW = PIPE_WAVES(W);
	constexpr int NT = 64 * NW;
	constexpr int CPP = W / 16;
	constexpr int ROWDW = W / 4 + 1;
	constexpr bool PORTS = (FEAT & (F_UDP | F_TCP)) != 0;
	constexpr uint32_t HIT = (FEAT & F_DENY) ? A_PASS : A_DROP;
	constexpr uint32_t MISS = (FEAT & F_DENY) ? A_DROP : A_PASS;
	constexpr uint32_t QTAG = 0x80000000u;   // tag bit: a QT slot (hit log), not a counter identity
	static_assert(NW * 64 * ROWDW * 4 >= 64 * XFG_QT_BUCKET * NW, "buckets fit the rows");
	__shared__ uint32_t win[NW * 64 * ROWDW > LOG_SCRATCH ? NW * 64 * ROWDW : LOG_SCRATCH];
	__shared__ uint32_t s_tab[PORTS ? XFG_PORT_TAB : 1];
	__shared__ uint32_t s_pcnt[PORTS ? XFG_PORT_TAB : 1];
	__shared__ uint32_t s_ctag[CC_ENTRIES], s_ccnt[CC_ENTRIES], s_tn[NW];
	__shared__ uint32_t s_lh[XFG_LOG_PARTS];
	__shared__ unsigned long long s_stats[6];
	extern __shared__ uint32_t s_dyn[];

	const int tid = threadIdx.x, lane = tid & 63;
	const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
	// the index, in scalar registers
	const uint64_t qb = rfl64((uint64_t)(uintptr_t)a.qt);
	const uint32_t qbits = rfl(a.qt_bits), qseed = rfl(a.qt_seed);
	const uint32_t rsh = 32 - qbits, rmask = (1u << rsh) - 1;
	const bool dlive = a.qt_live == M_DST;   // the one live key: dst (else src)
	const bool klive = a.t4.count != 0;
	Counters cn{ s_ctag, s_ccnt, dcnt_base(a, s_dyn) };
	cn.init(a, tid, NT);
	if (tid < 6)
		s_stats[tid] = 0;
	const uint32_t *s_ports = stage_ports<FEAT>(a, s_tab, s_dyn, tid, NT);
	const bool ptab = PORTS && a.port_count && a.port_tab;
	const uint32_t pdisp = rfl(a.port_tab_disp), gb3 = rfl(a.gbase[3]);
	if constexpr (PORTS)
		for (int i = tid; i < (int)XFG_PORT_TAB; i += NT)
			s_pcnt[i] = 0;
	for (int i = tid; i < (int)XFG_LOG_PARTS; i += NT)
		s_lh[i] = 0;
	__syncthreads();

	uint32_t *const rows = win + wv * 64 * ROWDW;
	const uint32_t *const myrow = rows + lane * ROWDW;
	uint32_t *const dlist = reinterpret_cast<uint32_t *>(
		rfl64((uint64_t)(uintptr_t)(a.defer + ((uint64_t)blockIdx.x * NW + wv) * a.defer_cap)));
	uint32_t *const tregion = reinterpret_cast<uint32_t *>(
		rfl64((uint64_t)(uintptr_t)(a.tlog + ((uint64_t)blockIdx.x * NW + wv) * a.defer_cap)));
	uint32_t tn = 0;
	// a hit's counter: a QT slot to the hit log (the host runs this kernel
	// only with the log on); a ruled port's to its table slot's LDS
	// counter; any other (the deferred packets') through Counters::bump
	auto count = [&](uint32_t tag, uint32_t pslot) {
		const bool q = (tag != CT_NONE) & ((tag & QTAG) != 0);
		const bool ps = pslot < XFG_PORT_TAB;
		const bool dc = !q & (tag < a.dcnt);
		const uint32_t qs = tag & ~QTAG;
		log_append(tregion, tn, pick(q, qs, CT_NONE), lane);
		if (q)
			atomicAdd(&s_lh[log_part(qs)], 1u);
		if constexpr (PORTS)
			if (ps)
				atomicAdd(&s_pcnt[pslot], 1u);
		if (dc & !ps)
			atomicAdd(&cn.dcnt[tag], 1u);
		cn.bump(a, pick(q | dc | ps, CT_NONE, tag), lane);
	};
	const uint32_t n = (uint32_t)a.n;
	const uint32_t nt = (n + 63) / 64;
	const uint32_t first = blockIdx.x * NW + wv;
	const uint32_t step = gridDim.x * NW;
	uint32_t st_c0 = 0, st_c1 = 0, st_c2 = 0, st_b0 = 0, st_b1 = 0, st_b2 = 0;
	auto stat = [&](uint32_t act, uint32_t len) {
		st_c0 += (uint32_t)__popcll(__ballot(act == A_ABORTED));
		st_c1 += (uint32_t)__popcll(__ballot(act == A_DROP));
		st_c2 += (uint32_t)__popcll(__ballot(act == A_PASS));
		st_b0 += pick(act == A_ABORTED, len, 0u);
		st_b1 += pick(act == A_DROP, len, 0u);
		st_b2 += pick(act == A_PASS, len, 0u);
	};
	uint32_t ndef = 0;

	// windows + lengths of tile t (clamped to the last tile): CPP + 2 loads,
	// always issued (as xfg_pipe4_kernel's)
	const bool l16 = a.lens_u16 != 0;
	const uint32_t lsh = l16 ? 1u : 2u;
	const uint64_t lb = rfl64((uint64_t)(uintptr_t)a.lens);
	auto issue = [&](uint32_t t, u32x4 (&pre)[CPP], uint16_t (&plen)[2]) {
		t = t < nt ? t : nt - 1;
		const uint32_t base = t * 64;
		const uint32_t rem = n - base >= 64 ? 64u : n - base;
#pragma unroll
		for (int it = 0; it < CPP; it++) {
			const uint32_t c = it * 64 + lane, pk = c / CPP, sub = c % CPP;
			const uint32_t q = pk < rem ? pk : 0u;
			const u32x4 *src = DENSE ? reinterpret_cast<const u32x4 *>(a.data + (uint64_t)base * W) + (q * CPP + sub)
						 : reinterpret_cast<const u32x4 *>(a.data + (uint64_t)(base + q) * a.stride + sub * 16);
			pre[it] = __builtin_nontemporal_load(src);
		}
		const uint64_t la = lb + ((uint64_t)(base + ((uint32_t)lane < rem ? lane : 0u)) << lsh);
		plen[0] = *reinterpret_cast<const __attribute__((address_space(1))) uint16_t *>(la);
		plen[1] = *reinterpret_cast<const __attribute__((address_space(1))) uint16_t *>(la + (lsh - 1) * 2);
	};

	auto pk3 = [](uint32_t act, uint32_t ps, uint32_t len) { return act | ps << 3 | len << 15; };
	auto pk_act = [](uint32_t p) { return p & 7; };
	auto pk_ps = [](uint32_t p) { return (p >> 3) & 0xfff; };
	auto pk_len = [](uint32_t p) { return p >> 15; };
	// P -> R (tile k-1): remainder, bucket, fallback
	uint32_t r_rem = 0, r_b = 0, r_pk = pk3(A_NONE, XFG_PORT_TAB, 0), r_tag = CT_NONE;
	bool r_sel = false;

	auto iteration = [&](uint32_t k, u32x4 (&cur)[CPP], uint16_t (&curlen)[2]) {
		const uint32_t tP = first + k * step;
		const bool vP = tP < nt;
		const bool vR = k >= 1 && tP - step < nt;
		__builtin_amdgcn_s_waitcnt(0x0F70 | ((CPP + 2) & 15) | (((CPP + 2) >> 4) << 14));
		asm volatile("" ::: "memory");   // (the LDS-DMA'd buckets: read only after the wait)

		// ---- R: tile k-1's bucket -> CHECK_MAP (xdpfilt_prog.h:56-64)
		const uint32_t r_act = pk_act(r_pk), r_ps = pk_ps(r_pk), w_len = pk_len(r_pk);
		uint32_t w_act = A_NONE, w_tag = CT_NONE, w_ps = r_ps;
		if (vR) {
			// packet p's bucket: halves at (p>>5)*1024 + (j*32 + (p&31))*16 bytes
			const u32x4 *bp4 = reinterpret_cast<const u32x4 *>(rows) + (lane >> 5) * 64 + (lane & 31);
			const u32x4 h0 = bp4[0], h1 = bp4[32];
			const uint32_t w[8] = { h0.x, h0.y, h0.z, h0.w, h1.x, h1.y, h1.z, h1.w };
			const uint32_t rr = r_rem | (r_rem << 16);
			uint32_t mm = 0, lv = 0;
#pragma unroll
			for (int i = 0; i < 8; i++) {
				// zero 15-bit halves of (w ^ rr): bit 15 / 31 of ~t (no borrow
				// crosses the halves: each is at least 0x7fff after the -1)
				const uint32_t z = (w[i] ^ rr) & 0x7fff7fffu;
				const uint32_t t = ~((z | 0x80008000u) - 0x00010001u) & 0x80008000u;
				const uint32_t v = t >> 15, l = (w[i] & 0x80008000u) >> 15;
				mm |= ((v | (v >> 15)) & 3u) << (2 * i);
				lv |= ((l | (l >> 15)) & 3u) << (2 * i);
			}
			const uint32_t cntq = w[0] & 15;
			mm &= ((2u << cntq) - 2u) & 0xfffeu;   // entries 1..count
			const bool found = r_sel & (mm != 0);
			const bool hit = found & ((mm & lv) != 0);
			const bool defer = r_sel & !found & ((w[0] & XFG_QT_OVF) != 0);
			const uint32_t slot = r_b * XFG_QT_SLOTS + (uint32_t)__builtin_ctz(mm | 0x10000u) - 1;
			w_act = pick(hit, HIT, pick(defer, A_DEFER, r_act));
			w_tag = pick(hit, QTAG | slot, pick(defer, CT_NONE, r_tag));
			w_ps = pick(hit | defer, XFG_PORT_TAB, r_ps);
		}

		// ---- W: verdicts, counters, stats, deferrals of tile k-1
		if (vR) {
			const uint32_t gi = (tP - step) * 64 + lane;
			if (w_act <= A_PASS)
				__builtin_nontemporal_store((uint8_t)w_act, a.verdicts + gi);
			count(w_tag, w_ps);
			stat(w_act, w_len);
			const unsigned long long dm = __ballot(w_act == A_DEFER);
			if (dm) {
				const uint32_t pos = ndef + lanes_below(dm);
				if (w_act == A_DEFER)
					gst32(dlist + pos, gi);
				ndef += (uint32_t)__popcll(dm);
			}
		}

		// ---- S: tile k's windows into the rows (past the batch's end:
		// zeroes), lengths clamped to the stride
		uint32_t len = 0;
		if (vP) {
			const uint32_t rem = n - tP * 64 >= 64 ? 64u : n - tP * 64;
			__builtin_amdgcn_wave_barrier();
#pragma unroll
			for (int it = 0; it < CPP; it++) {
				const int c = it * 64 + lane;
				const int pk = c / CPP, sub = c % CPP;
				const bool ok = (uint32_t)pk < rem;
				uint32_t *dst = &rows[pk * ROWDW + sub * 4];
				dst[0] = ok ? cur[it].x : 0u;
				dst[1] = ok ? cur[it].y : 0u;
				dst[2] = ok ? cur[it].z : 0u;
				dst[3] = ok ? cur[it].w : 0u;
			}
			const uint32_t l = l16 ? (uint32_t)curlen[0] : (uint32_t)curlen[0] | (uint32_t)curlen[1] << 16;
			len = (uint32_t)lane < rem ? min(l, a.stride) : 0u;
			__builtin_amdgcn_wave_barrier();
		}

		// ---- P: parse tile k, hash its key, plan its fallback
		bool lsel = false;
		if (vP) {
			const uint32_t gi = tP * 64 + lane;
			const Parse4 r = parse_bf<FEAT, W>(myrow, len);
			const bool valid = gi < n;
			const bool kok = valid & !r.defer & r.v4ok & klive;
			const uint32_t key = dlive ? r.k4a : r.k4b;
			const uint32_t h = xfg_qt_hash(key, qseed);
			r_b = h >> rsh;
			r_rem = h & rmask;
			r_sel = kok;
			lsel = kok;
			uint32_t fa = pick(r.abort_at != NST, A_ABORTED, MISS), ft = CT_NONE, fs = XFG_PORT_TAB;
			if constexpr (PORTS) {
				if (a.port_count) {
					const uint32_t pm = pick(r.l4proto == 17, M_UDP, M_TCP);
					const uint32_t pfm = a.port_fmask;
					bool ph = false;
					if (can_hit(pfm, M_DST)) {
						uint32_t sl;
						const uint32_t f = port_probe(s_ports, ptab, pdisp, r.pdst, sl);
						const uint32_t mk = M_DST | pm;
						ph = (r.l4proto != 0) & ((f & mk) == mk) & can_hit(pfm, mk);
						ft = pick(ph, gb3 + r.pdst, ft);
						fs = pick(ph, sl, fs);
					}
					if (can_hit(pfm, M_SRC)) {
						uint32_t sl;
						const uint32_t f = port_probe(s_ports, ptab, pdisp, r.psrc, sl);
						const uint32_t mk = M_SRC | pm;
						const bool h2 = !ph & (r.l4proto != 0) & ((f & mk) == mk) & can_hit(pfm, mk);
						ft = pick(h2, gb3 + r.psrc, ft);
						fs = pick(h2, sl, fs);
						ph |= h2;
					}
					fa = pick(ph, HIT, fa);
				}
			}
			r_pk = pk3(pick(!valid, A_NONE, pick(r.defer, A_DEFER, fa)),
				   pick(valid & !r.defer, fs, XFG_PORT_TAB), len);
			r_tag = pick(valid & !r.defer, ft, CT_NONE);
		} else {
			r_sel = false;
			r_pk = pk3(A_NONE, XFG_PORT_TAB, 0);
			r_tag = CT_NONE;
		}

		// ---- L: tile k's buckets LDS-DMA'd into the rows (free once P has
		// read them): instruction q carries packets 32q..32q+31, lane L the
		// 16-byte half L >> 5 of packet 32q + (L & 31)'s bucket
		{
			const unsigned long long need = __ballot(lsel);
			if (need) {
				__builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0): P's row reads are done
				__builtin_amdgcn_sched_barrier(0);
#pragma unroll
				for (int q = 0; q < 2; q++) {
					const uint32_t p = q * 32 + (lane & 31);
					const uint32_t bp = __shfl(r_b, (int)p);
					if ((need >> p) & 1)
						__builtin_amdgcn_global_load_lds(
							(const __attribute__((address_space(1))) void *)(
								qb + (uint64_t)bp * XFG_QT_BUCKET + (lane >> 5) * 16),
							(__attribute__((address_space(3))) void *)(rows + q * 256), 16, 0, 0);
				}
			}
		}
		// ---- tile k+2's windows, last: in flight for two iterations
		__builtin_amdgcn_sched_barrier(0);
		issue(tP + 2 * step, cur, curlen);
		__builtin_amdgcn_sched_barrier(0);
	};

	u32x4 preA[CPP], preB[CPP];
	uint16_t lenA[2] = { 0, 0 }, lenB[2] = { 0, 0 };
	if (nt) {
		issue(first, preA, lenA);
		__builtin_amdgcn_sched_barrier(0);
		issue(first + step, preB, lenB);
		__builtin_amdgcn_sched_barrier(0);
	}
	const uint32_t iters = first < nt ? (nt - 1 - first) / step + 2 : 0u;
	uint32_t k = 0;
	for (; k + 1 < iters; k += 2) {
		iteration(k, preA, lenA);
		iteration(k + 1, preB, lenB);
	}
	if (k < iters)
		iteration(k, preA, lenA);

#ifdef XFG_DIAG
	// (diagnostics: 2048 skips the deferred packets -- results wrong)
	if (a.diag & 2048)
		ndef = 0;
#endif
	// the deferred packets: the whole reference walk over the canonical
	// table (classify_staged), 64 at a time
	for (uint32_t d0 = 0; d0 < ndef; d0 += 64) {
		uint32_t act = A_NONE, tag = CT_NONE, len = 0;
		const bool ok = d0 + lane < ndef;
		const uint32_t gi = ok ? gld32(dlist + d0 + lane) : 0u;
		if (ok)
			len = min(load_len(a, gi), a.stride);
		act = classify_staged<FEAT, W>(a, s_ports, const_cast<uint32_t *>(myrow), ok, gi, len, tag);
		if (ok)
			__builtin_nontemporal_store((uint8_t)act, a.verdicts + gi);
		count(tag, XFG_PORT_TAB);
		stat(act, len);
	}

	const uint32_t vb[3] = { st_b0, st_b1, st_b2 }, vc[3] = { st_c0, st_c1, st_c2 };
#pragma unroll
	for (int kk = 0; kk < 3; kk++) {
		unsigned long long x = vb[kk];
#pragma unroll
		for (int o = 32; o > 0; o >>= 1)
			x += __shfl_xor(x, o);
		if (lane == 0 && vc[kk]) {
			atomicAdd(&s_stats[2 * kk], (unsigned long long)vc[kk]);
			atomicAdd(&s_stats[2 * kk + 1], x);
		}
	}
	if (lane == 0)
		s_tn[wv] = tn;
	__syncthreads();
	if (tid < 6 && s_stats[tid])
		atomicAdd(&a.stats[tid], s_stats[tid]);
	cn.flush(a, tid, NT);
	if constexpr (PORTS)
		if (ptab)
			for (int i = tid; i < (int)XFG_PORT_TAB; i += NT)
				if (s_pcnt[i])
					atomicAdd(a.port_hits + (s_tab[i] & 0xffff), (unsigned long long)s_pcnt[i]);
#ifdef XFG_DIAG
	if (a.diag & 16)   // (diagnostics: no workgroup-end partition -- counts wrong)
		return;
#endif
	if (a.tlog)   // (win is free now: the partition scratch)
		log_partition<NW>(a, s_tn, s_lh, win, tid);
}

}  // namespace
