/* tools/xfsynth.c — seeded synthetic traffic for tests and bench.py.
 *
 * Bench/test tooling, not part of the classifier.  Two generators, both
 * driven by xorshift64* so every run with the same seed is byte-identical:
 *
 *  xfs_gen_workload(): the BASELINE.json configurations:
 *     C2  64 B IPv4/UDP, a fraction of dst IPs drawn from the rule set;
 *     C3  64 B mix 80% IPv4/UDP, 10% IPv4/TCP (doff 5), 10% IPv6/UDP (62 B),
 *         ~1% malformed frames of the Appendix A classes;
 *     C4  IMIX 64/570/1514 in a 7:4:1 ratio, same header mix as C3;
 *     C5  1514 B frames, same header mix as C3.
 *  xfs_gen_fuzz(): structured random frames over every branch of the parser
 *     (VLAN stacks, IPv4 options/ihl, ARP, IPv6 extension chains, ICMPv6
 *     NDISC, UDP/TCP) followed by random truncation and field corruption,
 *     with addresses/ports drawn from the rule pools so lookups hit.
 */
#include <stdint.h>
#include <string.h>

struct rng { uint64_t s; };

static inline uint64_t rnext(struct rng *r)
{
	uint64_t x = r->s;
	x ^= x >> 12;
	x ^= x << 25;
	x ^= x >> 27;
	r->s = x;
	return x * 0x2545F4914F6CDD1Dull;
}
static inline uint32_t r32(struct rng *r) { return (uint32_t)(rnext(r) >> 32); }
static inline uint32_t rbelow(struct rng *r, uint32_t n) { return (uint32_t)(((uint64_t)r32(r) * n) >> 32); }
static inline int rchance(struct rng *r, uint32_t permille) { return rbelow(r, 1000) < permille; }

static inline void put16(uint8_t *p, uint32_t v) { p[0] = v >> 8; p[1] = v & 0xff; }

struct pools {
	const uint8_t *v4; uint32_t n4;   /* 4-byte keys */
	const uint8_t *v6; uint32_t n6;   /* 16-byte keys */
	const uint8_t *mac; uint32_t nm;  /* 6-byte keys */
	const uint16_t *ports; uint32_t np; /* port numbers (host order) */
};

static void rand_bytes(struct rng *r, uint8_t *p, uint32_t n)
{
	for (uint32_t i = 0; i < n; i++)
		p[i] = (uint8_t)rnext(r);
}

static void mac_rand(struct rng *r, uint8_t *p)
{
	rand_bytes(r, p, 6);
	p[0] = (p[0] & 0xfc) | 0x02; /* locally administered unicast */
}

static void pick_v4(struct rng *r, const struct pools *pl, uint32_t permille, uint8_t *p)
{
	if (pl->n4 && rchance(r, permille))
		memcpy(p, pl->v4 + 4ull * rbelow(r, pl->n4), 4);
	else
		rand_bytes(r, p, 4);
}

static void pick_v6(struct rng *r, const struct pools *pl, uint32_t permille, uint8_t *p)
{
	if (pl->n6 && rchance(r, permille))
		memcpy(p, pl->v6 + 16ull * rbelow(r, pl->n6), 16);
	else
		rand_bytes(r, p, 16);
}

static uint32_t pick_port(struct rng *r, const struct pools *pl, uint32_t permille)
{
	if (pl->np && rchance(r, permille))
		return pl->ports[rbelow(r, pl->np)];
	return r32(r) & 0xffff;
}

/* Writes L4 header at p (UDP or TCP); returns header bytes. */
static uint32_t put_l4(struct rng *r, const struct pools *pl, uint8_t *p, int tcp,
		       uint32_t l4len, uint32_t port_permille)
{
	put16(p + 0, pick_port(r, pl, port_permille / 4));
	put16(p + 2, pick_port(r, pl, port_permille));
	if (tcp) {
		memset(p + 4, 0, 16);
		p[12] = 5 << 4;  /* doff = 5 */
		p[13] = 0x10;    /* ACK */
		return 20;
	}
	put16(p + 4, l4len);
	p[6] = p[7] = 0;
	return 8;
}

static uint32_t put_ipv4(uint8_t *p, uint32_t proto, uint32_t totlen)
{
	p[0] = 0x45; p[1] = 0;
	put16(p + 2, totlen);
	p[4] = p[5] = 0; p[6] = 0x40; p[7] = 0; /* DF */
	p[8] = 64; p[9] = (uint8_t)proto;
	p[10] = p[11] = 0;
	return 20;
}

static void put_ipv6(uint8_t *p, uint32_t nexthdr, uint32_t paylen)
{
	p[0] = 0x60; p[1] = p[2] = p[3] = 0;
	put16(p + 4, paylen);
	p[6] = (uint8_t)nexthdr; p[7] = 64;
}

/* One well-formed frame of the workload mix (cls 0 IPv4/UDP, 1 IPv4/TCP,
 * 2 IPv6/UDP) of total length len (>= minimum for the class). */
static uint32_t gen_good(struct rng *r, const struct pools *pl, uint8_t *p, int cls,
			 uint32_t len, uint32_t dst_permille, uint32_t port_permille)
{
	mac_rand(r, p);
	mac_rand(r, p + 6);
	if (cls == 2) {
		put16(p + 12, 0x86DD);
		put_ipv6(p + 14, 17, len - 54);
		pick_v6(r, pl, dst_permille / 4, p + 22);     /* saddr */
		pick_v6(r, pl, dst_permille, p + 38);         /* daddr */
		put_l4(r, pl, p + 54, 0, len - 54, port_permille);
		return 62;
	}
	put16(p + 12, 0x0800);
	put_ipv4(p + 14, cls == 1 ? 6 : 17, len - 14);
	rand_bytes(r, p + 26, 4);                      /* saddr: random */
	pick_v4(r, pl, dst_permille, p + 30);          /* daddr */
	return 34 + put_l4(r, pl, p + 34, cls == 1, len - 34, port_permille);
}

/* Malformed frames of SURVEY.md Appendix A, all within 64 bytes. */
static uint32_t gen_bad(struct rng *r, const struct pools *pl, uint8_t *p, uint32_t maxlen)
{
	uint32_t kind = rbelow(r, 8), len = 64 < maxlen ? 64 : maxlen;
	gen_good(r, pl, p, 0, len, 500, 250);
	switch (kind) {
	case 0: return 13;                                  /* runt */
	case 1: p[38] = 0; p[39] = 7; return len;           /* UDP len 7 */
	case 2: return 41;                                  /* truncated UDP */
	case 3: p[14] = 0x4f; return len;                   /* ihl 15 > frame */
	case 4: put16(p + 12, 0x0806); memset(p + 14, 0, 28); return 42;  /* zero ARP */
	case 5: put16(p + 12, 0x86DD); put_ipv6(p + 14, 17, 0); return 54; /* IPv6, no L4 */
	case 6: put16(p + 12, 0x8100); return 16;           /* truncated VLAN */
	default: put16(p + 12, 0x88cc); return len;         /* LLDP */
	}
}

/* C1 (BASELINE.json configs[0]): a 64 B Ethernet/IPv4/UDP
 * frame whose MACs are random except that with probability @hit_permille
 * one ruled MAC is placed where its rule tests it: rule i of the 8 in the
 * destination MAC for i < 4 (the dst rules), in the source MAC for i >= 4
 * (the src rules).  @macs: the 8 ruled MACs, 6 bytes each. */
static void gen_c1(struct rng *r, const struct pools *pl, uint8_t *p, uint32_t hit_permille)
{
	gen_good(r, pl, p, 0, 64, 0, 0);
	if (pl->nm && rchance(r, hit_permille)) {
		const uint32_t i = rbelow(r, pl->nm);
		memcpy(p + (i < pl->nm / 2 ? 0 : 6), pl->mac + 6ull * i, 6);
	}
}

/* Workload generator.  kind: 1 = C1 (MAC pool in @v6 as 6-byte keys, @n6 of
 * them; dst_permille = the ruled-MAC fraction), 2 = C2, 3 = C3, 4 = C4 (IMIX),
 * 5 = C5 (1514).
 * Frames are written at data + i*stride (stride >= the largest frame).
 * dst_permille: fraction (x1000) of IPv4/IPv6 dst addresses drawn from the
 * rule pools.  Returns 0, or -1 if stride is too small. */
int xfs_gen_workload(uint64_t seed, int kind, uint64_t n, uint32_t stride,
		     uint8_t *data, uint32_t *lens,
		     const uint8_t *v4, uint32_t n4, const uint8_t *v6, uint32_t n6,
		     const uint16_t *ports, uint32_t np, uint32_t dst_permille,
		     uint32_t port_permille, uint32_t bad_permille)
{
	struct pools pl = { v4, n4, v6, n6, NULL, 0, ports, np };
	if (kind == 1) {   /* C1: the MAC pool rides in the v6 arguments */
		pl.mac = v6;
		pl.nm = n6;
		pl.v6 = NULL;
		pl.n6 = 0;
	}
	static const uint32_t imix[12] = { 64, 64, 64, 64, 64, 64, 64, 570, 570, 570, 570, 1514 };
	uint32_t need = kind == 4 || kind == 5 ? 1514 : 64;
	if (stride < need)
		return -1;
	for (uint64_t i = 0; i < n; i++) {
		struct rng r = { (seed + 1) * 0x9E3779B97F4A7C15ull ^ (i * 0xD1B54A32D192ED03ull) };
		uint8_t *p = data + i * (uint64_t)stride;
		uint32_t len, cls;
		rnext(&r);
		if (kind == 4)
			len = imix[rbelow(&r, 12)];
		else if (kind == 5)
			len = 1514;
		else
			len = 64;
		if (kind == 1 || kind == 2) {
			cls = 0;
		} else {
			uint32_t c = rbelow(&r, 10);
			cls = c < 8 ? 0 : (c == 8 ? 1 : 2);
		}
		if (bad_permille && rchance(&r, bad_permille)) {
			memset(p, 0, need < stride ? need : stride);
			lens[i] = gen_bad(&r, &pl, p, len);
			continue;
		}
		if (kind == 1) {
			gen_c1(&r, &pl, p, dst_permille);
			for (uint32_t o = 42; o < len; o++)
				p[o] = (uint8_t)(o * 7 + i);
			lens[i] = len;
			continue;
		}
		if (cls == 2 && len == 64)
			len = 62; /* IPv6/UDP header-only frame, 2 B pad */
		gen_good(&r, &pl, p, cls, len, dst_permille, port_permille);
		/* payload bytes: deterministic filler (not parsed) */
		for (uint32_t o = (cls == 2 ? 62 : (cls == 1 ? 54 : 42)); o < len; o++)
			p[o] = (uint8_t)(o * 7 + i);
		lens[i] = len;
	}
	return 0;
}

/* ---------------- structured fuzz ---------------------------------------- */
static const uint8_t ext_types[6] = { 0, 60, 43, 135, 51, 44 };

static uint32_t fuzz_one(struct rng *r, const struct pools *pl, uint8_t *p, uint32_t cap)
{
	uint32_t o = 12, cls = rbelow(r, 12);
	uint32_t ethertype;
	if (pl->nm && rchance(r, 200))
		memcpy(p, pl->mac + 6ull * rbelow(r, pl->nm), 6);
	else
		mac_rand(r, p);
	if (pl->nm && rchance(r, 150))
		memcpy(p + 6, pl->mac + 6ull * rbelow(r, pl->nm), 6);
	else
		mac_rand(r, p + 6);
	/* VLAN stack: 0..5 tags (the 5th is beyond VLAN_MAX_DEPTH) */
	if (rchance(r, 250)) {
		uint32_t tags = rbelow(r, 6);
		for (uint32_t t = 0; t < tags; t++) {
			put16(p + o, rchance(r, 500) ? 0x8100 : 0x88A8);
			put16(p + o + 2, r32(r) & 0xfff);
			o += 4;
		}
	}
	switch (cls) {
	case 0: ethertype = rchance(r, 500) ? 0x88cc : (r32(r) & 0xffff); break;
	case 1: case 2: case 3: case 4: ethertype = 0x0800; break;
	case 5: ethertype = 0x0806; break;
	default: ethertype = 0x86DD; break;
	}
	put16(p + o, ethertype);
	o += 2;
	uint32_t len = o;
	if (ethertype == 0x0800) {
		uint32_t proto = cls == 1 ? 17 : cls == 2 ? 6 : cls == 3 ? 1 : (rchance(r, 500) ? 17 : 6);
		uint32_t ihl = rchance(r, 850) ? 5 : rbelow(r, 16);
		put_ipv4(p + o, proto, 0);
		p[o] = 0x40 | ihl;
		if (rchance(r, 100)) p[o + 6] = 0x20; /* MF: fragments are accepted */
		rand_bytes(r, p + o + 12, 4);
		pick_v4(r, pl, 400, p + o + 12);
		pick_v4(r, pl, 400, p + o + 16);
		uint32_t hl = ihl * 4 < 20 ? 20 : ihl * 4;
		if (hl > 20) rand_bytes(r, p + o + 20, hl - 20);
		uint32_t l4 = o + ihl * 4;  /* may overlap the IP header (ihl < 5) */
		if (proto == 17 || proto == 6) {
			uint32_t tcp = proto == 6;
			if (l4 + 20 + 16 > cap) l4 = o + 20;
			put_l4(r, pl, p + l4, tcp, 8 + rbelow(r, 64), 500);
			if (tcp && rchance(r, 150)) p[l4 + 12] = (uint8_t)(rbelow(r, 16) << 4);
			if (!tcp && rchance(r, 100)) put16(p + l4 + 4, rbelow(r, 10));
			len = (l4 > o + hl ? l4 : o + hl) + (tcp ? 20 : 8) + rbelow(r, 24);
		} else {
			len = o + hl + rbelow(r, 32);
		}
	} else if (ethertype == 0x0806) {
		put16(p + o, rchance(r, 900) ? 1 : r32(r) & 3);
		put16(p + o + 2, rchance(r, 900) ? 0x0800 : 0x86DD);
		p[o + 4] = rchance(r, 900) ? 6 : (uint8_t)rbelow(r, 8);
		p[o + 5] = rchance(r, 900) ? 4 : (uint8_t)rbelow(r, 8);
		put16(p + o + 6, rbelow(r, 4));
		mac_rand(r, p + o + 8);
		pick_v4(r, pl, 400, p + o + 14);
		mac_rand(r, p + o + 18);
		pick_v4(r, pl, 400, p + o + 24);
		len = o + 28 + rbelow(r, 8);
	} else if (ethertype == 0x86DD) {
		uint32_t nexts = rchance(r, 500) ? 0 : rbelow(r, 7);
		uint32_t final = cls == 6 ? 17 : cls == 7 ? 6 : cls == 8 ? 58 : cls == 9 ? 58 : (r32(r) & 0xff);
		uint32_t cur = o + 40;
		put_ipv6(p + o, nexts ? ext_types[rbelow(r, 6)] : final, 0);
		pick_v6(r, pl, 400, p + o + 8);
		pick_v6(r, pl, 400, p + o + 24);
		uint32_t nh = p[o + 6];
		for (uint32_t e = 0; e < nexts && cur + 16 < cap; e++) {
			uint32_t next = e + 1 < nexts ? ext_types[rbelow(r, 6)] : final;
			uint32_t hlen = rbelow(r, 3), sz;
			p[cur] = (uint8_t)next;
			p[cur + 1] = (uint8_t)hlen;
			if (nh == 51) sz = (hlen + 2) * 4;
			else if (nh == 44) sz = 8;
			else sz = (hlen + 1) * 8;
			if (cur + sz + 40 > cap) { p[cur + 1] = 0; sz = nh == 51 ? 8 : 8; }
			if (sz > 2) rand_bytes(r, p + cur + 2, sz - 2);
			p[cur] = (uint8_t)next;
			cur += sz;
			nh = next;
		}
		if (final == 17 || final == 6) {
			put_l4(r, pl, p + cur, final == 6, 8 + rbelow(r, 32), 500);
			len = cur + (final == 6 ? 20 : 8) + rbelow(r, 16);
		} else if (final == 58) {
			p[cur] = rchance(r, 700) ? (rchance(r, 500) ? 135 : 136) : (uint8_t)r32(r);
			p[cur + 1] = 0;
			memset(p + cur + 2, 0, 6);
			pick_v6(r, pl, 500, p + cur + 8);
			len = cur + 24 + rbelow(r, 8);
		} else {
			len = cur + rbelow(r, 16);
		}
	} else {
		len = o + rbelow(r, 32);
	}
	if (len > cap) len = cap;
	/* random truncation / corruption */
	if (rchance(r, 120))
		len = rbelow(r, len + 1);
	if (rchance(r, 40)) {
		uint32_t k = rbelow(r, len ? len : 1);
		if (len) p[k] ^= (uint8_t)(1u << rbelow(r, 8));
	}
	return len;
}

/* Fuzz generator: frames at data + i*stride (stride >= 128), length in lens.
 * Pools provide keys that rules exist for, so lookups frequently hit. */
int xfs_gen_fuzz(uint64_t seed, uint64_t n, uint32_t stride, uint8_t *data, uint32_t *lens,
		 const uint8_t *v4, uint32_t n4, const uint8_t *v6, uint32_t n6,
		 const uint8_t *mac, uint32_t nm, const uint16_t *ports, uint32_t np)
{
	struct pools pl = { v4, n4, v6, n6, mac, nm, ports, np };
	if (stride < 128)
		return -1;
	for (uint64_t i = 0; i < n; i++) {
		struct rng r = { (seed + 7) * 0x9E3779B97F4A7C15ull ^ (i * 0xD1B54A32D192ED03ull) };
		uint8_t *p = data + i * (uint64_t)stride;
		rnext(&r);
		rand_bytes(&r, p, stride);
		lens[i] = fuzz_one(&r, &pl, p, stride);
	}
	return 0;
}

/* Random distinct-ish keys: n keys of keylen bytes (seeded). */
void xfs_rand_keys(uint64_t seed, uint64_t n, uint32_t keylen, uint8_t *out)
{
	struct rng r = { (seed + 3) * 0x9E3779B97F4A7C15ull | 1 };
	for (uint64_t i = 0; i < n * keylen; i++)
		out[i] = (uint8_t)rnext(&r);
}
