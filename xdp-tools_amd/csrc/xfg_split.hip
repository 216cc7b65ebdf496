// SPDX-License-Identifier: GPL-2.0
//
// xfg_split.hip — the IPv4-key classify (key mode 1: only IPv4 keys can hit,
// by the flag census) as two kernels.  Included by xfg_kernels.hip after
// xfg_pipeline.hip, whose parse and lookup helpers it shares.
//
// xfg_pipe4_kernel runs the stream, the parse and the dependent lookup hops
// in one wave, so every wait for a Bloom word or a bucket line is also a
// wait for the frame loads issued before it (a wave's vector-memory counter
// completes in issue order), and the random lookups are issued while the
// stream holds the memory queues.  Here the two halves run apart:
//
//   xfg_parse4_kernel  the HBM-bound half: frames streamed with coalesced
//                      16-byte loads, staged in LDS rows, parsed (the same
//                      branch-free parse of the common shapes, parse_bf);
//                      per packet a record: a state byte (in the verdict
//                      buffer), the first live IPv4 key, the L4 ports and,
//                      when both directions are live, the second key.
//   xfg_look4_kernel   the latency-bound half: records in, Bloom word, bucket
//                      line (LDS-DMA), CHECK_MAP (xdpfilt_prog.h:56-64), the
//                      port stage (:76-101, from LDS), verdict, counters,
//                      stats, deferred packets -- the R/W/Q/L stages of
//                      xfg_pipe4_kernel with nothing else in the wave's queue.
//
// Results are those of xfg_pipe4_kernel, bit for bit: same parse, same key
// order, same deferral rules, same counting.
namespace {

// Record state byte (written to the packet's verdict byte by the parse pass,
// replaced by its verdict in the lookup pass).
constexpr uint32_t SB_DEFER = 1, SB_ABORT = 2, SB_UDP = 4, SB_TCP = 8, SB_KA = 16, SB_KB = 32;

constexpr int PARSE_WAVES = 4;

typedef __attribute__((address_space(1))) uint32_t gw32;
typedef __attribute__((address_space(1))) uint8_t gw8;

template <uint32_t FEAT, int W, bool DENSE>
__global__ __launch_bounds__(64 * PARSE_WAVES) void xfg_parse4_kernel(const xfg_kargs a)
{
	static_assert((FEAT & F_IPV4) != 0, "IPv4-key mode needs the IPv4 feature");
	constexpr int NW = PARSE_WAVES;
	constexpr int CPP = W / 16;
	constexpr int ROWDW = W / 4 + 1;
	__shared__ uint32_t win[NW * 64 * ROWDW];

	const int tid = threadIdx.x, lane = tid & 63;
	const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
	uint32_t *const rows = win + wv * 64 * ROWDW;
	const uint32_t *const myrow = rows + lane * ROWDW;
	const bool dlive = a.t4.count && can_hit(a.t4.fmask, M_DST);
	const bool slive = a.t4.count && can_hit(a.t4.fmask, M_SRC);
	const bool both = dlive & slive;
	const uint32_t n = (uint32_t)a.n;
	const uint32_t nt = (n + 63) / 64;
	const uint32_t first = blockIdx.x * NW + wv;
	const uint32_t step = gridDim.x * NW;
	const bool l16 = a.lens_u16 != 0;
	const uint32_t lsh = l16 ? 1u : 2u;
	const uint64_t lb = rfl64((uint64_t)(uintptr_t)a.lens);
	// a length is one dword load: the aligned word holding it (one load
	// instruction for both widths; two 16-bit loads get packed into one
	// register right after issue, which waits for them there)
	auto len_word = [&](uint32_t i) { return (lb + ((uint64_t)i << lsh)) & ~3ull; };
	auto len_of = [&](uint32_t w, uint32_t i) {
		return l16 ? (w >> (((lb + ((uint64_t)i << 1)) & 2) * 8)) & 0xffffu : w;
	};
	gw8 *const vout = reinterpret_cast<gw8 *>(rfl64((uint64_t)(uintptr_t)a.verdicts));
	gw32 *const ka_out = reinterpret_cast<gw32 *>(rfl64((uint64_t)(uintptr_t)a.rec_ka));
	gw32 *const kb_out = reinterpret_cast<gw32 *>(rfl64((uint64_t)(uintptr_t)a.rec_kb));
	gw32 *const pt_out = reinterpret_cast<gw32 *>(rfl64((uint64_t)(uintptr_t)a.rec_port));

	// windows + lengths of tile t into one of two register sets (lanes past
	// the batch's end read a valid address; the staging zeroes them)
	auto issue = [&](uint32_t t, u32x4 (&pre)[CPP], uint32_t &plen) {
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
		plen = gload32(len_word(base + ((uint32_t)lane < rem ? lane : 0u)));
	};
	// the previous tile's record, stored after the next tile's loads are out
	uint32_t o_st = 0, o_ka = 0, o_kb = 0, o_pt = 0, o_gi = 0;
	bool o_ok = false;
	auto put = [&]() {
		if (o_ok) {
			vout[o_gi] = (uint8_t)o_st;
			ka_out[o_gi] = o_ka;
			pt_out[o_gi] = o_pt;
			if (both)
				kb_out[o_gi] = o_kb;
		}
	};
	// One tile: its windows (in `cur`, issued an iteration ago) staged and
	// parsed while tile t + 2 step's go out into the same registers.  Two
	// register sets alternate (the loop is unrolled by two), so no copy of
	// an in-flight load ever waits at the end of an iteration.
	auto iteration = [&](uint32_t t, u32x4 (&cur)[CPP], uint32_t &curlen) {
		// everything but the other set's loads (issued last iteration)
		__builtin_amdgcn_s_waitcnt(0x0F70 | ((CPP + 1) & 15) | (((CPP + 1) >> 4) << 14));
		const uint32_t rem = n - t * 64 >= 64 ? 64u : n - t * 64;
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
		const uint32_t len = (uint32_t)lane < rem ? min(len_of(curlen, t * 64 + lane), a.stride) : 0u;
		__builtin_amdgcn_wave_barrier();
		put();
		const uint32_t gi = t * 64 + lane;
		const Parse4 r = parse_bf<FEAT, W>(myrow, len);
		const bool kok = !r.defer & r.v4ok;
		const bool ka = kok & (dlive | slive);
		const bool kb = kok & both;
		o_ka = dlive ? r.k4a : r.k4b;
		o_kb = r.k4b;
		o_pt = r.pdst | r.psrc << 16;
		o_st = pick(r.defer, SB_DEFER,
			    pick(r.abort_at != NST, SB_ABORT, 0u) | pick(r.l4proto == 17, SB_UDP, 0u) |
				    pick(r.l4proto == 6, SB_TCP, 0u) | pick(ka, SB_KA, 0u) | pick(kb, SB_KB, 0u));
		o_gi = gi;
		o_ok = gi < n;
		// tile t + 2 step's windows, last (clamped: a fixed load count)
		__builtin_amdgcn_sched_barrier(0);
		const uint32_t tn = t + 2 * step;
		issue(tn < nt ? tn : nt - 1, cur, curlen);
		__builtin_amdgcn_sched_barrier(0);
	};

	u32x4 preA[CPP], preB[CPP];
	uint32_t lenA = 0, lenB = 0;
	if (first >= nt)
		return;
	issue(first, preA, lenA);
	__builtin_amdgcn_sched_barrier(0);
	issue(first + step < nt ? first + step : nt - 1, preB, lenB);
	__builtin_amdgcn_sched_barrier(0);
	uint32_t t = first;
	for (; t + step < nt; t += 2 * step) {
		iteration(t, preA, lenA);
		iteration(t + step, preB, lenB);
	}
	if (t < nt)
		iteration(t, preA, lenA);
	put();
}

// Lookup pass.  One wave works alone on tiles of 64 packets (one per lane),
// three tiles one hop apart, one wait per iteration (as xfg_pipe4_kernel):
//   R(k-2) match the bucket lines -> verdict, counter identity
//   W(k-2) verdicts, counters, stats, deferrals
//   Q(k-1) Bloom words -> the first candidate key and its bucket
//   P(k)   records -> the port-stage fallback, hashes, Bloom words issued
//   L(k-1) candidate bucket lines, LDS-DMA'd into the wave's area
//   I      tile k+2's records issued, last
template <uint32_t FEAT, int W>
__global__ __launch_bounds__(PIPE_THREADS(W), 4) void xfg_look4_kernel(const xfg_kargs a)
{
	constexpr int NW = PIPE_WAVES(W);
	constexpr int NT = 64 * NW;
	constexpr int ROWDW = W / 4 + 1;
	// per wave: 64 bucket lines, or the deferred packets' window rows
	constexpr int AREA = 64 * ROWDW > 1024 ? 64 * ROWDW : 1024;
	constexpr bool PORTS = (FEAT & (F_UDP | F_TCP)) != 0;
	constexpr uint32_t HIT = (FEAT & F_DENY) ? A_PASS : A_DROP;
	constexpr uint32_t MISS = (FEAT & F_DENY) ? A_DROP : A_PASS;
	// record loads per tile: state, key a, key b, length, and the ports
	// when the program has an L4 stage (the wait below counts on exactly
	// these being the iteration's last vector-memory instructions)
	constexpr int NR = PORTS ? 5 : 4;
	__shared__ uint32_t win[NW * AREA > LOG_SCRATCH ? NW * AREA : LOG_SCRATCH];
	__shared__ uint32_t s_tab[PORTS ? XFG_PORT_TAB : 1];
	__shared__ uint32_t s_pcnt[PORTS ? XFG_PORT_TAB : 1];
	__shared__ uint32_t s_ctag[CC_ENTRIES], s_ccnt[CC_ENTRIES], s_tn[NW];
	__shared__ uint32_t s_lh[XFG_LOG_PARTS];
	__shared__ unsigned long long s_stats[6];
	extern __shared__ uint32_t s_dyn[];

	const int tid = threadIdx.x, lane = tid & 63;
	const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
	const uint32_t nb = rfl(a.t4.nbuckets), md = rfl(a.t4.max_disp), ns = rfl(a.t4.nslots);
	const uint32_t zp = rfl(a.t4.zero_present), bw = rfl(a.t4.bloom_words);
	const uint32_t seed = rfl(a.t4.seed), gb = rfl(a.gbase[0]), gb3 = rfl(a.gbase[3]);
	const uint64_t bk = rfl64((uint64_t)(uintptr_t)a.t4.buckets);
	const uint64_t bl = rfl64((uint64_t)(uintptr_t)a.t4.bloom);
	const bool dlive = a.t4.count && can_hit(a.t4.fmask, M_DST);
	const bool slive = a.t4.count && can_hit(a.t4.fmask, M_SRC);
	const bool both = dlive & slive;
	const uint32_t mask_a = dlive ? M_DST : M_SRC;
	// without a prefilter every live key goes to its bucket line (one key
	// per packet only: the host sets bloom_off only then)
	const bool nobloom = a.bloom_off != 0;
#ifdef XFG_DIAG
	const uint32_t dg = a.diag;
#else
	constexpr uint32_t dg = 0;
#endif
	Counters cn{ s_ctag, s_ccnt, dcnt_base(a, s_dyn) };
	cn.init(a, tid, NT);
	if (tid < 6)
		s_stats[tid] = 0;
	const uint32_t *s_ports = stage_ports<FEAT>(a, s_tab, s_dyn, tid, NT);
	const bool ptab = PORTS && a.port_count && a.port_tab;
	const uint32_t pdisp = rfl(a.port_tab_disp);
	if constexpr (PORTS)
		for (int i = tid; i < (int)XFG_PORT_TAB; i += NT)
			s_pcnt[i] = 0;
	for (int i = tid; i < (int)XFG_LOG_PARTS; i += NT)
		s_lh[i] = 0;
	__syncthreads();

	uint32_t *const rows = win + wv * AREA;
	uint32_t *const myrow = rows + lane * ROWDW;
	uint32_t *const dlist = reinterpret_cast<uint32_t *>(
		rfl64((uint64_t)(uintptr_t)(a.defer + ((uint64_t)blockIdx.x * NW + wv) * a.defer_cap)));
	uint32_t *const tregion = reinterpret_cast<uint32_t *>(
		rfl64((uint64_t)(uintptr_t)(a.tlog + ((uint64_t)blockIdx.x * NW + wv) * a.defer_cap)));
	uint32_t tn = 0;
	const uint32_t lg_lo = rfl(a.dcnt), lg_hi = a.tlog ? rfl(a.gbase[3]) : 0u;
	auto count = [&](uint32_t tag, uint32_t pslot) {
		const bool ps = pslot < XFG_PORT_TAB;
		const bool dc = tag < lg_lo;
		const bool lg = (tag >= lg_lo) & (tag < lg_hi);
		log_append(tregion, tn, pick(lg, tag, CT_NONE), lane);
		if (lg)
			atomicAdd(&s_lh[log_part(tag)], 1u);
		if constexpr (PORTS)
			if (ps)
				atomicAdd(&s_pcnt[pslot], 1u);
		if (dc & !ps)
			atomicAdd(&cn.dcnt[tag], 1u);
		cn.bump(a, pick(lg | dc | ps, CT_NONE, tag), lane);
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

	// records of tile t (clamped to the last tile): NR loads, always issued
	const bool l16 = a.lens_u16 != 0;
	const uint32_t lsh = l16 ? 1u : 2u;
	const uint64_t lb = rfl64((uint64_t)(uintptr_t)a.lens);
	const uint64_t vb = rfl64((uint64_t)(uintptr_t)a.verdicts);
	const uint64_t rka = rfl64((uint64_t)(uintptr_t)a.rec_ka);
	const uint64_t rkb = both ? rfl64((uint64_t)(uintptr_t)a.rec_kb) : rka;
	const uint64_t rpt = rfl64((uint64_t)(uintptr_t)a.rec_port);
	auto len_word = [&](uint64_t i) { return (lb + (i << lsh)) & ~3ull; };
	auto issue = [&](uint32_t t, uint32_t (&rc)[4], uint32_t &rl) {
		t = t < nt ? t : nt - 1;
		const uint32_t base = t * 64;
		const uint32_t rem = n - base >= 64 ? 64u : n - base;
		const uint64_t i = base + ((uint32_t)lane < rem ? lane : 0u);
		rc[0] = *reinterpret_cast<const gw8 *>(vb + i);
		rc[1] = gload32(rka + 4 * i);
		rc[2] = 0;
		if constexpr (PORTS)
			rc[2] = gload32(rpt + 4 * i);
		rc[3] = gload32(rkb + 4 * i);
		rl = gload32(len_word(i));
	};

	auto pk3 = [](uint32_t act, uint32_t ps, uint32_t len) { return act | ps << 3 | len << 15; };
	auto pk_act = [](uint32_t p) { return p & 7; };
	auto pk_ps = [](uint32_t p) { return (p >> 3) & 0xfff; };
	auto pk_len = [](uint32_t p) { return p >> 15; };
	// P -> Q (tile k-1)
	uint32_t q_ka = 0, q_kb = 0, q_wa = 0, q_wb = 0, q_f = 0;
	uint32_t q_pk = pk3(A_NONE, XFG_PORT_TAB, 0), q_tag = CT_NONE;
	// Q -> R (tile k-2)
	uint32_t r_key = 0, r_b = 0, r_mask = 0, r_pk = pk3(A_NONE, XFG_PORT_TAB, 0), r_tag = CT_NONE;
	bool r_sel = false, r_zero = false, r_more = false;

	auto iteration = [&](uint32_t k, uint32_t (&rc)[4], uint32_t &rl) {
		const uint32_t tP = first + k * step;
		const bool vP = tP < nt;
		const bool vQ = k >= 1 && tP - step < nt;
		const bool vR = k >= 2 && tP - 2 * step < nt;
		// the one wait: everything but the newest tile's records
		__builtin_amdgcn_s_waitcnt(0x0F70 | (NR & 15) | ((NR >> 4) << 14));
		asm volatile("" ::: "memory");

		// ---- R: CHECK_MAP on tile k-2's lines
		const uint32_t r_act = pk_act(r_pk), r_ps = pk_ps(r_pk), w_len = pk_len(r_pk);
		uint32_t w_act = A_NONE, w_tag = CT_NONE, w_ps = r_ps;
		if (vR) {
			Line r_line;
			{
				const u32x4 *lp4 = reinterpret_cast<const u32x4 *>(rows) + lane * 4;
				r_line.q0 = lp4[0];
				r_line.q1 = lp4[1];
				r_line.q2 = lp4[2];
				r_line.q3 = lp4[3];
			}
			const int m = match_v4(r_line, r_key);
			const bool found = r_zero | (m >= 0);
			const uint32_t i = pick(r_zero | (m < 0), 0u, (uint32_t)m);
			const uint32_t fl = r_line.flag((int)i);
			const bool hit = r_sel & found & ((fl & r_mask) == r_mask);
			const uint32_t slot = pick(r_zero, ns, r_b * XFG_SLOTS_V4 + i);
			const bool defer = r_sel & !hit & (r_more | (!found & r_line.overflow() & (md != 0)));
			w_act = pick(hit, HIT, pick(defer, A_DEFER, r_act));
			w_tag = pick(hit, gb + slot, pick(defer, CT_NONE, r_tag));
			w_ps = pick(hit | defer, XFG_PORT_TAB, r_ps);
		}

		// ---- W: tile k-2's verdicts, counters, stats, deferrals
		if (vR) {
			const uint32_t gi = (tP - 2 * step) * 64 + lane;
			if (w_act <= A_PASS && !(dg & 8))
				__builtin_nontemporal_store((uint8_t)w_act, a.verdicts + gi);
			count((dg & 1) ? CT_NONE : w_tag, (dg & 1) ? XFG_PORT_TAB : w_ps);
			stat(w_act, w_len);
			const unsigned long long dm = __ballot(w_act == A_DEFER);
			if (dm) {
				const uint32_t pos = ndef + lanes_below(dm);
				if (w_act == A_DEFER)
					gst32(dlist + pos, gi);
				ndef += (uint32_t)__popcll(dm);
			}
		}

		// ---- Q: tile k-1's Bloom words -> first candidate key, its bucket
		bool lsel = false;
		if (vQ) {
			const uint32_t q_ha = xfg_hash_v4(q_ka, seed), q_hb = xfg_hash_v4(q_kb, seed);
			const uint32_t bma = xfg_bloom_mask(q_ha), bmb = xfg_bloom_mask(q_hb);
			const bool za = (q_f & KF_AZ) != 0, zb = (q_f & KF_BZ) != 0;
			const bool ma = ((q_f & KF_A) != 0) & (za ? zp != 0 : (nobloom | ((q_wa & bma) == bma)));
			const bool mb = ((q_f & KF_B) != 0) & (zb ? zp != 0 : (q_wb & bmb) == bmb);
			r_sel = ma | mb;
			r_more = ma & mb;
			r_key = pick(ma, q_ka, q_kb);
			r_zero = ma ? za : zb;
			r_mask = pick(ma, mask_a, M_SRC);
			r_b = pick(r_zero, nb, xfg_home(pick(ma, q_ha, q_hb), nb));
			r_pk = q_pk;
			r_tag = q_tag;
			lsel = r_sel;
		}

		// ---- P: tile k's records -> keys, fallback; Bloom words issued
		if (vP) {
			const uint32_t gi = tP * 64 + lane;
			const bool valid = gi < n;
			const uint32_t s = rc[0];
			const bool defer = (s & SB_DEFER) != 0;
			const uint32_t l = l16 ? (rl >> (((lb + ((uint64_t)gi << 1)) & 2) * 8)) & 0xffffu : rl;
			const uint32_t len = valid ? min(l, a.stride) : 0u;
			const bool ka = valid & ((s & SB_KA) != 0);
			const bool kb = valid & ((s & SB_KB) != 0);
			q_ka = rc[1];
			q_kb = rc[3];
			const uint32_t q_ha = xfg_hash_v4(q_ka, seed), q_hb = xfg_hash_v4(q_kb, seed);
			q_f = pick(ka, KF_A, 0u) | pick(kb, KF_B, 0u) | pick(q_ka == 0, KF_AZ, 0u) |
			      pick(q_kb == 0, KF_BZ, 0u);
			const uint32_t l4proto = pick((s & SB_UDP) != 0, 17u, pick((s & SB_TCP) != 0, 6u, 0u));
			const uint32_t pdst = rc[2] & 0xffff, psrc = rc[2] >> 16;
			uint32_t fa = pick((s & SB_ABORT) != 0, A_ABORTED, MISS), ft = CT_NONE, fs = XFG_PORT_TAB;
			if constexpr (PORTS) {
				if (a.port_count) {
					const uint32_t pm = pick(l4proto == 17, M_UDP, M_TCP);
					const uint32_t pfm = a.port_fmask;
					bool ph = false;
					if (can_hit(pfm, M_DST)) {
						uint32_t sl;
						const uint32_t f = port_probe(s_ports, ptab, pdisp, pdst, sl);
						const uint32_t mk = M_DST | pm;
						ph = (l4proto != 0) & ((f & mk) == mk) & can_hit(pfm, mk);
						ft = pick(ph, gb3 + pdst, ft);
						fs = pick(ph, sl, fs);
					}
					if (can_hit(pfm, M_SRC)) {
						uint32_t sl;
						const uint32_t f = port_probe(s_ports, ptab, pdisp, psrc, sl);
						const uint32_t mk = M_SRC | pm;
						const bool h = !ph & (l4proto != 0) & ((f & mk) == mk) & can_hit(pfm, mk);
						ft = pick(h, gb3 + psrc, ft);
						fs = pick(h, sl, fs);
						ph |= h;
					}
					fa = pick(ph, HIT, fa);
				}
			}
			q_pk = pk3(pick(!valid, A_NONE, pick(defer, A_DEFER, fa)),
				   pick(valid & !defer, fs, XFG_PORT_TAB), len);
			q_tag = pick(valid & !defer, ft, CT_NONE);
			q_wa = q_wb = ~0u;
			if ((q_f & (KF_A | KF_AZ)) == KF_A && !nobloom && !(dg & 4))
				q_wa = gload32(bl + 4ull * xfg_bloom_word(q_ha, bw));
			if ((q_f & (KF_B | KF_BZ)) == KF_B && !(dg & 4))
				q_wb = gload32(bl + 4ull * xfg_bloom_word(q_hb, bw));
		}

		// ---- L: tile k-1's candidate lines into the wave's area
		// (instruction q carries packets 16q..16q+15, four lanes a line)
		{
			const unsigned long long need = __ballot(lsel && !(dg & 2));
			if (need) {
				__builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0): R's reads are done
				__builtin_amdgcn_sched_barrier(0);
#pragma unroll
				for (int q = 0; q < 4; q++) {
					const uint32_t p = q * 16 + (lane >> 2);
					const uint32_t pj = lane & 3;
					const uint32_t bp = __shfl(r_b, (int)p);
					if ((need >> p) & 1)
						__builtin_amdgcn_global_load_lds(
							(const __attribute__((address_space(1))) void *)(
								bk + (uint64_t)bp * XFG_BUCKET_BYTES + pj * 16),
							(__attribute__((address_space(3))) void *)(rows + q * 256), 16, 0, 0);
				}
			}
		}
		// ---- tile k+2's records, last
		__builtin_amdgcn_sched_barrier(0);
		issue(tP + 2 * step, rc, rl);
		__builtin_amdgcn_sched_barrier(0);
	};

	uint32_t rcA[4], rcB[4];
	uint32_t rlA = 0, rlB = 0;
	if (nt) {
		issue(first, rcA, rlA);
		__builtin_amdgcn_sched_barrier(0);
		issue(first + step, rcB, rlB);
		__builtin_amdgcn_sched_barrier(0);
	}
	const uint32_t iters = first < nt ? (nt - 1 - first) / step + 3 : 0u;
	uint32_t k = 0;
	for (; k + 1 < iters; k += 2) {
		iteration(k, rcA, rlA);
		iteration(k + 1, rcB, rlB);
	}
	if (k < iters)
		iteration(k, rcA, rlA);

	// deferred packets: the whole reference program over the staged window
	for (uint32_t d0 = 0; d0 < ndef; d0 += 64) {
		uint32_t act = A_NONE, tag = CT_NONE, len = 0;
		const bool ok = d0 + lane < ndef;
		const uint32_t gi = ok ? gld32(dlist + d0 + lane) : 0u;
		if (ok)
			len = min(load_len(a, gi), a.stride);
		act = classify_staged<FEAT, W>(a, s_ports, myrow, ok, gi, len, tag);
		if (ok)
			__builtin_nontemporal_store((uint8_t)act, a.verdicts + gi);
		count(tag, XFG_PORT_TAB);
		stat(act, len);
	}

	const uint32_t vbs[3] = { st_b0, st_b1, st_b2 }, vcs[3] = { st_c0, st_c1, st_c2 };
#pragma unroll
	for (int kk = 0; kk < 3; kk++) {
		unsigned long long x = vbs[kk];
#pragma unroll
		for (int o = 32; o > 0; o >>= 1)
			x += __shfl_xor(x, o);
		if (lane == 0 && vcs[kk]) {
			atomicAdd(&s_stats[2 * kk], (unsigned long long)vcs[kk]);
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
	if (a.tlog && !(dg & 16))   // (win is free now: the partition scratch)
		log_partition<NW>(a, s_tn, s_lh, win, tid);
}

}  // namespace
