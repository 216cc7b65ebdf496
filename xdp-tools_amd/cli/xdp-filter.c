/* SPDX-License-Identifier: GPL-2.0 */
/*
 * xdp-filter — the command line of the MI355X classifier.
 *
 * Same commands, options, rule semantics and output format as the reference
 * CLI (xdp-filter/xdp-filter.c, command table :1104-1114), over the C ABI of
 * libxdpfilter_gpu.so instead of libbpf/libxdp:
 *
 *   load    select the program exactly as find_prog_file() does (:48-60) and
 *           "pin" its maps: create the map files of the rule store
 *           (include/xdpfilter_io.h) and record the program for <ifname>
 *   unload  drop the record; remove maps no loaded program uses (:357-431)
 *   port / ip / ether
 *           map_get_counter_flags() / map_set_flags() (:73-157) on the
 *           stored maps, through a host-only xfg context
 *   status / poll
 *           the readouts of :965-1083 and lib/util/stats.c:48-292
 *   run     (no reference counterpart: the kernel attach is replaced) —
 *           classify a pcap/pcapng capture as traffic arriving on <ifname>
 *           on the GPUs, update the stored hit counters and per-action
 *           stats, optionally dump a pcapng with per-packet XDP verdicts
 *
 * The state directory ($XDP_FILTER_STATE_DIR, default /run/xdp-filter-gpu)
 * takes the place of /sys/fs/bpf/xdp-filter; a flock on <dir>/.lock takes
 * the place of prog_lock_acquire() (lib/util/util.c:727-767).
 */
#define _GNU_SOURCE
#include <arpa/inet.h>
#include <dirent.h>
#include <errno.h>
#include <fcntl.h>
#include <inttypes.h>
#include <locale.h>
#include <pthread.h>
#include <signal.h>
#include <stdarg.h>
#include <stdbool.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/file.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include "xdpfilter_gpu.h"
#include "xdpfilter_io.h"

#define PROG_NAME "xdp-filter"
#define MAP_FLAGS (XFG_MAP_FLAG_SRC | XFG_MAP_FLAG_DST | XFG_MAP_FLAG_TCP | XFG_MAP_FLAG_UDP)

/* ------------------------------------------------------------------ logging */
static int verbose;

static void pr(int level, const char *fmt, ...)
{
	va_list ap;
	if (level > verbose)
		return;
	va_start(ap, fmt);
	vfprintf(stderr, fmt, ap);
	va_end(ap);
}
#define pr_warn(...) pr(0, __VA_ARGS__)
#define pr_info(...) pr(0, __VA_ARGS__)
#define pr_debug(...) pr(1, __VA_ARGS__)

/* ------------------------------------------------------------------ flags */
struct flag_val {
	const char *s;
	unsigned v;
};

static const struct flag_val map_flags_all[] = {
	{ "src", XFG_MAP_FLAG_SRC }, { "dst", XFG_MAP_FLAG_DST },
	{ "tcp", XFG_MAP_FLAG_TCP }, { "udp", XFG_MAP_FLAG_UDP }, { 0, 0 } };
static const struct flag_val map_flags_srcdst[] = {
	{ "src", XFG_MAP_FLAG_SRC }, { "dst", XFG_MAP_FLAG_DST }, { 0, 0 } };
static const struct flag_val map_flags_tcpudp[] = {
	{ "tcp", XFG_MAP_FLAG_TCP }, { "udp", XFG_MAP_FLAG_UDP }, { 0, 0 } };
static const struct flag_val load_features[] = {
	{ "tcp", XFG_FEAT_TCP }, { "udp", XFG_FEAT_UDP }, { "ipv6", XFG_FEAT_IPV6 },
	{ "ipv4", XFG_FEAT_IPV4 }, { "ethernet", XFG_FEAT_ETHERNET }, { "all", XFG_FEAT_ALL },
	{ 0, 0 } };
static const struct flag_val print_features[] = {
	{ "tcp", XFG_FEAT_TCP }, { "udp", XFG_FEAT_UDP }, { "ipv6", XFG_FEAT_IPV6 },
	{ "ipv4", XFG_FEAT_IPV4 }, { "ethernet", XFG_FEAT_ETHERNET },
	{ "allow", XFG_FEAT_ALLOW }, { "deny", XFG_FEAT_DENY }, { 0, 0 } };
static const struct flag_val xdp_modes[] = {
	{ "native", 0 }, { "skb", 1 }, { "hw", 2 }, { 0, 0 } };
static const struct flag_val policy_modes[] = {
	{ "allow", XFG_FEAT_ALLOW }, { "deny", XFG_FEAT_DENY }, { 0, 0 } };

/* "a,b,c" -> OR of the named flags (lib/util/params.c:217-239) */
static int parse_flags(const char *arg, const struct flag_val *fv, unsigned *out)
{
	char buf[256], *save = NULL, *tok;
	unsigned v = 0;
	snprintf(buf, sizeof(buf), "%s", arg);
	for (tok = strtok_r(buf, ",", &save); tok; tok = strtok_r(NULL, ",", &save)) {
		const struct flag_val *f;
		for (f = fv; f->s; f++)
			if (!strcmp(f->s, tok))
				break;
		if (!f->s)
			return -EINVAL;
		v |= f->v;
	}
	*out = v;
	return 0;
}

static int parse_enum(const char *arg, const struct flag_val *fv, unsigned *out)
{
	for (const struct flag_val *f = fv; f->s; f++)
		if (!strcmp(f->s, arg)) {
			*out = f->v;
			return 0;
		}
	return -EINVAL;
}

static const char *enum_name(const struct flag_val *fv, unsigned v)
{
	for (const struct flag_val *f = fv; f->s; f++)
		if (f->v == v)
			return f->s;
	return "unknown";
}

/* lib/util/params.c:401-425 */
static void print_flags(char *buf, size_t len, const struct flag_val *fv, unsigned set)
{
	size_t o = 0;
	buf[0] = '\0';
	for (const struct flag_val *f = fv; f->s; f++) {
		if (!(f->v & set))
			continue;
		int n = snprintf(buf + o, len - o, "%s%s", o ? "," : "", f->s);
		if (n < 0 || (size_t)n >= len - o)
			break;
		o += n;
	}
}

/* program table: name -> _features, xdp-filter/Makefile:3-6 order */
static const struct { const char *name; unsigned feat; } progs[] = {
	{ "xdpfilt_dny_udp", XFG_FEAT_UDP | XFG_FEAT_DENY },
	{ "xdpfilt_dny_tcp", XFG_FEAT_TCP | XFG_FEAT_DENY },
	{ "xdpfilt_dny_ip", XFG_FEAT_IPV4 | XFG_FEAT_IPV6 | XFG_FEAT_DENY },
	{ "xdpfilt_dny_eth", XFG_FEAT_ETHERNET | XFG_FEAT_DENY },
	{ "xdpfilt_dny_all", XFG_FEAT_ALL | XFG_FEAT_DENY },
	{ "xdpfilt_alw_udp", XFG_FEAT_UDP | XFG_FEAT_ALLOW },
	{ "xdpfilt_alw_tcp", XFG_FEAT_TCP | XFG_FEAT_ALLOW },
	{ "xdpfilt_alw_ip", XFG_FEAT_IPV4 | XFG_FEAT_IPV6 | XFG_FEAT_ALLOW },
	{ "xdpfilt_alw_eth", XFG_FEAT_ETHERNET | XFG_FEAT_ALLOW },
	{ "xdpfilt_alw_all", XFG_FEAT_ALL | XFG_FEAT_ALLOW },
};

/* find_features() (xdp-filter.c:62-71) */
static unsigned find_features(const char *name)
{
	for (size_t i = 0; i < sizeof(progs) / sizeof(progs[0]); i++)
		if (!strcmp(progs[i].name, name))
			return progs[i].feat;
	return 0;
}

/* ------------------------------------------------------------------ state dir */
static char state_dir[4096];

static void init_state_dir(void)
{
	const char *d = getenv("XDP_FILTER_STATE_DIR");
	snprintf(state_dir, sizeof(state_dir), "%s", d && *d ? d : "/run/xdp-filter-gpu");
}

static int path_in(char *buf, size_t n, const char *sub)
{
	int r = snprintf(buf, n, "%s/%s", state_dir, sub);
	return r < 0 || (size_t)r >= n ? -ENAMETOOLONG : 0;
}

static int mkdir_p(const char *p)
{
	char tmp[4096];
	snprintf(tmp, sizeof(tmp), "%s", p);
	for (char *s = tmp + 1; *s; s++) {
		if (*s != '/')
			continue;
		*s = '\0';
		if (mkdir(tmp, 0700) && errno != EEXIST)
			return -errno;
		*s = '/';
	}
	if (mkdir(tmp, 0700) && errno != EEXIST)
		return -errno;
	return 0;
}

/* prog_lock_acquire(): flock on <dir>/.lock, creating the directory */
static int lock_acquire(bool create)
{
	char p[4200];
	int err;
	if (create && (err = mkdir_p(state_dir))) {
		pr_warn("Couldn't create state directory %s: %s\n", state_dir, strerror(-err));
		return err;
	}
	if ((err = path_in(p, sizeof(p), ".lock")))
		return err;
	int fd = open(p, O_RDWR | O_CREAT | O_CLOEXEC, 0600);
	if (fd < 0) {
		if (!create && errno == ENOENT)
			return -ENOENT;
		err = -errno;
		pr_warn("Couldn't open lock file %s: %s\n", p, strerror(-err));
		return err;
	}
	if (flock(fd, LOCK_EX)) {
		err = -errno;
		close(fd);
		return err;
	}
	return fd;
}

static void lock_release(int fd)
{
	if (fd >= 0) {
		flock(fd, LOCK_UN);
		close(fd);
	}
}

struct prog_rec {
	char ifname[256];
	char prog[64];
	char mode[16];
};

static int prog_path(char *buf, size_t n, const char *ifname)
{
	int r = snprintf(buf, n, "%s/programs/%s", state_dir, ifname);
	return r < 0 || (size_t)r >= n ? -ENAMETOOLONG : 0;
}

static int read_prog(const char *ifname, struct prog_rec *r)
{
	char p[4400];
	int err = prog_path(p, sizeof(p), ifname);
	if (err)
		return err;
	FILE *f = fopen(p, "r");
	if (!f)
		return -errno;
	memset(r, 0, sizeof(*r));
	snprintf(r->ifname, sizeof(r->ifname), "%s", ifname);
	int n = fscanf(f, "%63s %15s", r->prog, r->mode);
	fclose(f);
	return n == 2 && find_features(r->prog) ? 0 : -EINVAL;
}

/* iterate_pinned_programs(): every program record, sorted by interface */
static int list_progs(struct prog_rec **out, int *count)
{
	char p[4200];
	struct dirent **ents = NULL;
	int err = path_in(p, sizeof(p), "programs");
	*out = NULL;
	*count = 0;
	if (err)
		return err;
	int n = scandir(p, &ents, NULL, alphasort);
	if (n < 0)
		return errno == ENOENT ? 0 : -errno;
	struct prog_rec *v = calloc(n ? n : 1, sizeof(*v));
	int m = 0;
	for (int i = 0; i < n; i++) {
		if (v && ents[i]->d_name[0] != '.' && !read_prog(ents[i]->d_name, &v[m]))
			m++;
		free(ents[i]);
	}
	free(ents);
	if (!v)
		return -ENOMEM;
	*out = v;
	*count = m;
	return 0;
}

static unsigned used_features(void)
{
	struct prog_rec *v;
	int n;
	unsigned f = 0;
	if (list_progs(&v, &n))
		return 0;
	for (int i = 0; i < n; i++)
		f |= find_features(v[i].prog);
	free(v);
	return f;
}

/* Host-only context holding the stored maps (capacities as stored). */
static xfg_ctx *open_store(int *err_out)
{
	struct xfg_open_opts o;
	xfg_ctx *ctx = NULL;
	memset(&o, 0, sizeof(o));
	o.sz = sizeof(o);
	o.features = XFG_FEAT_ALL | XFG_FEAT_DENY;
	int64_t c;
	if ((c = xfg_store_map_capacity(state_dir, XFG_MAP_IPV4)) > 0)
		o.ipv4_capacity = (uint32_t)c;
	if ((c = xfg_store_map_capacity(state_dir, XFG_MAP_IPV6)) > 0)
		o.ipv6_capacity = (uint32_t)c;
	if ((c = xfg_store_map_capacity(state_dir, XFG_MAP_ETHERNET)) > 0)
		o.eth_capacity = (uint32_t)c;
	int err = xfg_open(&ctx, &o);
	if (!err)
		err = xfg_store_load(ctx, state_dir);
	if (err) {
		pr_warn("Couldn't load the rule store in %s: %s\n", state_dir, xfg_strerror(err));
		xfg_close(ctx);
		ctx = NULL;
	}
	*err_out = err;
	return ctx;
}

/* map_get_counter_flags() (xdp-filter.c:73-109), one value per stored key */
static int get_counter_flags(xfg_ctx *ctx, int map, const void *key, uint64_t *counter,
			     uint8_t *flags)
{
	uint64_t v;
	if (xfg_map_lookup(ctx, map, key, &v))
		return -ENOENT;
	if (!(v & MAP_FLAGS))
		return -ENOENT;
	*flags = v & MAP_FLAGS;
	*counter = v >> XFG_COUNTER_SHIFT;
	return 0;
}

/* map_set_flags() (xdp-filter.c:111-157) */
static int set_flags(xfg_ctx *ctx, int map, const void *key, uint8_t flags, bool delete_empty)
{
	uint64_t v;
	int err;
	if (xfg_map_lookup(ctx, map, key, &v)) {
		v = 0;
	} else if (!flags && delete_empty) {
		pr_debug("Deleting empty map value from flags %u\n", flags);
		err = xfg_map_delete(ctx, map, key);
		if (err)
			pr_warn("Couldn't delete value from state map: %s\n", strerror(-err));
		return err;
	}
	v = flags ? (v & ~(uint64_t)MAP_FLAGS) | (flags & MAP_FLAGS) : 0;
	pr_debug("Setting new map value %" PRIu64 " from flags %u\n", v, flags);
	err = xfg_map_update(ctx, map, key, &v);
	if (err) {
		if (err == -E2BIG)
			pr_warn("Couldn't add entry: state map is full\n");
		else
			pr_warn("Unable to update state map: %s\n", strerror(-err));
	}
	return err;
}

/* ------------------------------------------------------------------ printing */
static int print_ports(xfg_ctx *ctx)
{
	static uint32_t keys[XFG_PORT_MAP_ENTRIES];
	static uint64_t vals[XFG_PORT_MAP_ENTRIES];
	for (uint32_t k = 0; k < XFG_PORT_MAP_ENTRIES; k++)
		keys[k] = k;
	int64_t r = xfg_map_lookup_batch(ctx, XFG_MAP_PORTS, keys, XFG_PORT_MAP_ENTRIES, vals, NULL);
	if (r < 0)
		return (int)r;
	printf("Filtered ports:\n");
	printf("  %-40s Mode             Hit counter\n", "");
	for (uint32_t k = 0; k < XFG_PORT_MAP_ENTRIES; k++) {
		char buf[100];
		uint8_t flags = vals[k] & MAP_FLAGS;
		if (!flags)
			continue;
		print_flags(buf, sizeof(buf), map_flags_all, flags);
		printf("  %-40u %-15s  %" PRIu64 "\n", ntohs((uint16_t)k), buf,
		       vals[k] >> XFG_COUNTER_SHIFT);
	}
	return 0;
}

static int print_addrs(xfg_ctx *ctx, int map)
{
	uint8_t key[16], prev[16];
	const void *pk = NULL;
	const int kl = map == XFG_MAP_IPV6 ? 16 : map == XFG_MAP_IPV4 ? 4 : 6;
	for (;;) {
		char flagbuf[100], addrbuf[100];
		uint64_t counter;
		uint8_t flags;
		int err = xfg_map_get_next_key(ctx, map, pk, key);
		if (err == -ENOENT)
			break;
		if (err)
			return err;
		memcpy(prev, key, kl);
		pk = prev;
		if (get_counter_flags(ctx, map, key, &counter, &flags))
			continue;
		print_flags(flagbuf, sizeof(flagbuf), map_flags_srcdst, flags);
		if (map == XFG_MAP_ETHERNET)
			snprintf(addrbuf, sizeof(addrbuf), "%02x:%02x:%02x:%02x:%02x:%02x", key[0],
				 key[1], key[2], key[3], key[4], key[5]);
		else
			inet_ntop(map == XFG_MAP_IPV6 ? AF_INET6 : AF_INET, key, addrbuf,
				  sizeof(addrbuf));
		printf("  %-40s %-15s  %" PRIu64 "\n", addrbuf, flagbuf, counter);
	}
	return 0;
}

/* print_ips(): IPv6 then IPv4; -ENOENT when neither map is pinned */
static int print_ips(xfg_ctx *ctx)
{
	bool h6 = xfg_store_has_map(state_dir, XFG_MAP_IPV6);
	bool h4 = xfg_store_has_map(state_dir, XFG_MAP_IPV4);
	int err = 0;
	if (!h4 && !h6)
		return -ENOENT;
	printf("Filtered IP addresses:\n");
	printf("  %-40s Mode             Hit counter\n", "");
	if (h6 && (err = print_addrs(ctx, XFG_MAP_IPV6)))
		return err;
	if (h4)
		err = print_addrs(ctx, XFG_MAP_IPV4);
	return err;
}

static int print_ethers(xfg_ctx *ctx)
{
	printf("Filtered MAC addresses:\n");
	printf("  %-40s Mode             Hit counter\n", "");
	return print_addrs(ctx, XFG_MAP_ETHERNET);
}

static const char *action2str(int a)
{
	static const char *names[] = { "XDP_ABORTED", "XDP_DROP", "XDP_PASS", "XDP_TX",
				       "XDP_REDIRECT" };
	return a >= 0 && a < 5 ? names[a] : "XDP_UNKNOWN";
}

/* ------------------------------------------------------------------ options */
struct opt {
	const char *name;
	char short_opt;
	bool has_arg;
	int id;
};

#define MAXPOS 4
struct args {
	const char *pos[MAXPOS];
	int npos;
	const char *val[32];
	bool set[32];
};

static int parse_args(int argc, char **argv, const struct opt *opts, struct args *a,
		      const char *usage)
{
	memset(a, 0, sizeof(*a));
	for (int i = 1; i < argc; i++) {
		const char *s = argv[i];
		const struct opt *o = NULL;
		const char *inl = NULL;
		if (!strcmp(s, "-v") || !strcmp(s, "--verbose")) {
			verbose = 1;
			continue;
		}
		if (!strcmp(s, "-h") || !strcmp(s, "--help")) {
			fprintf(stderr, "%s", usage);
			return 1;
		}
		if (s[0] == '-' && s[1] == '-' && s[2]) {
			const char *eq = strchr(s + 2, '=');
			size_t l = eq ? (size_t)(eq - s - 2) : strlen(s + 2);
			for (const struct opt *p = opts; p->name; p++)
				if (strlen(p->name) == l && !strncmp(p->name, s + 2, l))
					o = p;
			inl = eq ? eq + 1 : NULL;
		} else if (s[0] == '-' && s[1] && !s[2]) {
			for (const struct opt *p = opts; p->name; p++)
				if (p->short_opt == s[1])
					o = p;
		} else {
			if (a->npos >= MAXPOS) {
				pr_warn("Too many arguments\n");
				return -EINVAL;
			}
			a->pos[a->npos++] = s;
			continue;
		}
		if (!o) {
			pr_warn("Unknown option: %s\n%s", s, usage);
			return -EINVAL;
		}
		a->set[o->id] = true;
		if (o->has_arg) {
			if (!inl) {
				if (i + 1 >= argc) {
					pr_warn("Option %s requires an argument\n", s);
					return -EINVAL;
				}
				inl = argv[++i];
			}
			a->val[o->id] = inl;
		}
	}
	return 0;
}

static int parse_u32(const char *s, uint32_t max, uint32_t *out)
{
	char *end;
	errno = 0;
	unsigned long v = strtoul(s, &end, 10);
	if (errno || *end || v > max)
		return -EINVAL;
	*out = (uint32_t)v;
	return 0;
}

/* ------------------------------------------------------------------ load */
enum { O_MODE, O_POLICY, O_FEATURES, O_CAPACITY, O_ALL, O_KEEP, O_REMOVE, O_PROTO, O_STATUS,
       O_INTERVAL, O_COUNT, O_GPUS, O_DUMP, O_REPEAT, O_QUIET };

static int do_load(int argc, char **argv)
{
	static const struct opt opts[] = {
		{ "mode", 'm', true, O_MODE }, { "policy", 'p', true, O_POLICY },
		{ "features", 'f', true, O_FEATURES }, { "capacity", 'c', true, O_CAPACITY },
		{ 0, 0, 0, 0 } };
	const char *usage =
		"Usage: xdp-filter load [options] <ifname>\n"
		"  -m, --mode <mode>         Load XDP program in <mode>; default native (valid values: native,skb,hw)\n"
		"  -p, --policy <policy>     Policy for unmatched packets; default allow (valid values: allow,deny)\n"
		"  -f, --features <feats>    Features to enable; default all (valid values: tcp,udp,ipv6,ipv4,ethernet,all)\n"
		"  -c, --capacity <n>        Entries per hash map (the reference's max_entries); default 10000\n"
		"  -v, --verbose             Enable verbose logging\n";
	struct args a;
	unsigned mode = 0, policy = XFG_FEAT_ALLOW, features = XFG_FEAT_ALL;
	uint32_t capacity = XFG_DEFAULT_MAP_CAPACITY;
	char featbuf[100];
	int err = parse_args(argc, argv, opts, &a, usage);
	if (err)
		return err > 0 ? 0 : 1;
	if (a.npos != 1) {
		pr_warn("Missing required parameter <ifname>\n%s", usage);
		return 1;
	}
	if ((a.set[O_MODE] && parse_enum(a.val[O_MODE], xdp_modes, &mode)) ||
	    (a.set[O_POLICY] && parse_enum(a.val[O_POLICY], policy_modes, &policy)) ||
	    (a.set[O_FEATURES] && parse_flags(a.val[O_FEATURES], load_features, &features)) ||
	    (a.set[O_CAPACITY] && (parse_u32(a.val[O_CAPACITY], 1u << 30, &capacity) || !capacity))) {
		pr_warn("Invalid option value\n%s", usage);
		return 1;
	}
	const char *ifname = a.pos[0];
	if (mode == 2) {
		pr_warn("xdp-filter does not support offloading.\n");
		return 1;
	}
	if (strchr(ifname, '/') || ifname[0] == '.' || strlen(ifname) >= 64) {
		pr_warn("Invalid interface name: %s\n", ifname);
		return 1;
	}
	int lock = lock_acquire(true);
	if (lock < 0)
		return 1;
	err = 1;
	unsigned used = used_features();
	if (policy == XFG_FEAT_DENY && (used & XFG_FEAT_ALLOW)) {
		pr_warn("xdp-filter is already loaded in allow policy mode. "
			"Unload before loading in deny mode.\n");
		goto out;
	} else if (policy == XFG_FEAT_ALLOW && (used & XFG_FEAT_DENY)) {
		pr_warn("xdp-filter is already loaded in deny policy mode. "
			"Unload before loading in allow mode.\n");
		goto out;
	}
	features |= policy;
	struct prog_rec r;
	if (!read_prog(ifname, &r)) {
		pr_warn("xdp-filter is already loaded on %s\n", ifname);
		goto out;
	}
	print_flags(featbuf, sizeof(featbuf), print_features, features);
	pr_debug("Looking for eBPF program with features %s\n", featbuf);
	const char *prog;
	uint32_t pfeat;
	if (xfg_select_program(features, &prog, &pfeat)) {
		pr_warn("Couldn't find an eBPF program with the requested feature set!\n");
		goto out;
	}
	pr_debug("Found prog '%s' matching feature set to be loaded on interface '%s'.\n", prog,
		 ifname);
	/* pin the program's maps (LIBBPF_PIN_BY_NAME: existing ones are reused) */
	int e = 0;
	if (pfeat & (XFG_FEAT_TCP | XFG_FEAT_UDP))
		e = e ? e : xfg_store_create_map(state_dir, XFG_MAP_PORTS, 0);
	if (pfeat & XFG_FEAT_IPV4)
		e = e ? e : xfg_store_create_map(state_dir, XFG_MAP_IPV4, capacity);
	if (pfeat & XFG_FEAT_IPV6)
		e = e ? e : xfg_store_create_map(state_dir, XFG_MAP_IPV6, capacity);
	if (pfeat & XFG_FEAT_ETHERNET)
		e = e ? e : xfg_store_create_map(state_dir, XFG_MAP_ETHERNET, capacity);
	struct xfg_stats_record st[XFG_ACTION_MAX];
	if (!e && xfg_store_stats_read(state_dir, st)) {
		memset(st, 0, sizeof(st));
		e = xfg_store_stats_write(state_dir, st);
	}
	char pdir[4200], pfile[4400];
	if (!e && !(e = path_in(pdir, sizeof(pdir), "programs")))
		e = mkdir_p(pdir);
	if (!e && !(e = prog_path(pfile, sizeof(pfile), ifname))) {
		FILE *f = fopen(pfile, "w");
		if (!f)
			e = -errno;
		else {
			fprintf(f, "%s %s\n", prog, enum_name(xdp_modes, mode));
			if (fclose(f))
				e = -EIO;
		}
	}
	if (e) {
		pr_warn("Couldn't attach XDP program on iface '%s': %s(%d)\n", ifname, strerror(-e), e);
		goto out;
	}
	err = 0;
out:
	lock_release(lock);
	return err;
}

/* ------------------------------------------------------------------ unload */
static int remove_unused_maps(unsigned features)
{
	int err = 0;
	if (!(features & (XFG_FEAT_TCP | XFG_FEAT_UDP)))
		err = err ? err : xfg_store_remove_map(state_dir, XFG_MAP_PORTS);
	if (!(features & XFG_FEAT_IPV4))
		err = err ? err : xfg_store_remove_map(state_dir, XFG_MAP_IPV4);
	if (!(features & XFG_FEAT_IPV6))
		err = err ? err : xfg_store_remove_map(state_dir, XFG_MAP_IPV6);
	if (!(features & XFG_FEAT_ETHERNET))
		err = err ? err : xfg_store_remove_map(state_dir, XFG_MAP_ETHERNET);
	if (!err && !features) {
		char p[4200];
		err = xfg_store_stats_remove(state_dir);
		if (!err && !path_in(p, sizeof(p), "programs")) {
			pr_debug("Removing program directory %s\n", p);
			if (rmdir(p) && errno != ENOENT)
				err = -errno;
		}
		if (!err && !path_in(p, sizeof(p), ".lock"))
			unlink(p);
		if (!err) {
			pr_debug("Removing pinning directory %s\n", state_dir);
			if (rmdir(state_dir) && errno != ENOENT)
				err = -errno;
		}
		if (err)
			pr_warn("Unable to rmdir: %s\n", strerror(-err));
	}
	return err;
}

static int do_unload(int argc, char **argv)
{
	static const struct opt opts[] = {
		{ "all", 'a', false, O_ALL }, { "keep-maps", 'k', false, O_KEEP }, { 0, 0, 0, 0 } };
	const char *usage = "Usage: xdp-filter unload [options] [ifname]\n"
			    "  -a, --all                 Unload from all interfaces\n"
			    "  -k, --keep-maps           Don't destroy unused maps after unloading\n"
			    "  -v, --verbose             Enable verbose logging\n";
	struct args a;
	int err = parse_args(argc, argv, opts, &a, usage);
	if (err)
		return err > 0 ? 0 : 1;
	int lock = lock_acquire(false);
	if (lock == -ENOENT) {
		if (a.set[O_ALL])
			return 0;
		pr_warn("xdp-filter is not loaded on %s\n", a.npos ? a.pos[0] : "");
		return 1;
	}
	if (lock < 0)
		return 1;
	err = 1;
	char p[4400];
	if (a.set[O_ALL]) {
		struct prog_rec *v;
		int n;
		if (!list_progs(&v, &n)) {
			for (int i = 0; i < n; i++) {
				char pb[100];
				print_flags(pb, sizeof(pb), print_features, find_features(v[i].prog));
				pr_debug("Removing XDP program with features %s from iface %s\n", pb,
					 v[i].ifname);
				if (!prog_path(p, sizeof(p), v[i].ifname))
					unlink(p);
			}
			free(v);
		}
	} else {
		struct prog_rec r;
		if (!a.npos) {
			pr_warn("Must specify ifname or --all\n");
			goto out;
		}
		if (read_prog(a.pos[0], &r)) {
			pr_warn("xdp-filter is not loaded on %s\n", a.pos[0]);
			goto out;
		}
		char pb[100];
		print_flags(pb, sizeof(pb), print_features, find_features(r.prog));
		pr_debug("Removing XDP program with features %s from iface %s\n", pb, r.ifname);
		if (prog_path(p, sizeof(p), r.ifname) || unlink(p)) {
			pr_warn("Removing XDP program on iface %s failed\n", r.ifname);
			goto out;
		}
	}
	if (a.set[O_KEEP]) {
		pr_debug("Not removing pinned maps because of --keep-maps option\n");
		err = 0;
		goto out;
	}
	unsigned feats = used_features();
	char fb[100];
	print_flags(fb, sizeof(fb), print_features, feats);
	pr_debug("Features still being used: %s\n", feats ? fb : "none");
	err = remove_unused_maps(feats) ? 1 : 0;
out:
	lock_release(lock);
	return err;
}

/* ------------------------------------------------------------------ port/ip/ether */
static int do_port(int argc, char **argv)
{
	static const struct opt opts[] = {
		{ "remove", 'r', false, O_REMOVE }, { "mode", 'm', true, O_MODE },
		{ "proto", 'p', true, O_PROTO }, { "status", 's', false, O_STATUS }, { 0, 0, 0, 0 } };
	const char *usage =
		"Usage: xdp-filter port [options] <port>\n"
		"  -r, --remove              Remove port instead of adding\n"
		"  -m, --mode <mode>         Filter mode; default dst (valid values: src,dst)\n"
		"  -p, --proto <proto>       Protocol to filter; default tcp,udp (valid values: tcp,udp)\n"
		"  -s, --status              Print status of filtered ports after changing\n";
	struct args a;
	unsigned mode = 0, proto = 0;
	uint32_t port;
	char modestr[100], protostr[100];
	int err = parse_args(argc, argv, opts, &a, usage);
	if (err)
		return err > 0 ? 0 : 1;
	if (a.npos != 1 || parse_u32(a.pos[0], 0xffff, &port) ||
	    (a.set[O_MODE] && parse_flags(a.val[O_MODE], map_flags_srcdst, &mode)) ||
	    (a.set[O_PROTO] && parse_flags(a.val[O_PROTO], map_flags_tcpudp, &proto))) {
		pr_warn("Invalid or missing parameter\n%s", usage);
		return 1;
	}
	int lock = lock_acquire(false);
	if (lock < 0 || !xfg_store_has_map(state_dir, XFG_MAP_PORTS)) {
		pr_warn("Couldn't find port filter map; is xdp-filter loaded "
			"with the right features (udp and/or tcp)?\n");
		lock_release(lock);
		return 1;
	}
	xfg_ctx *ctx = open_store(&err);
	if (!ctx) {
		lock_release(lock);
		return 1;
	}
	uint32_t key = htons((uint16_t)port);
	uint8_t flags = 0;
	uint64_t counter;
	get_counter_flags(ctx, XFG_MAP_PORTS, &key, &counter, &flags);
	if (a.set[O_REMOVE]) {
		if (mode == 0 && proto == 0) {
			mode = XFG_MAP_FLAG_SRC | XFG_MAP_FLAG_DST;
			proto = XFG_MAP_FLAG_TCP | XFG_MAP_FLAG_UDP;
		}
		flags &= ~(mode | proto);
	} else {
		if (mode == 0)
			mode = XFG_MAP_FLAG_DST;
		if (proto == 0)
			proto = XFG_MAP_FLAG_TCP | XFG_MAP_FLAG_UDP;
		flags |= mode | proto;
	}
	print_flags(modestr, sizeof(modestr), map_flags_srcdst, mode);
	print_flags(protostr, sizeof(protostr), map_flags_tcpudp, proto);
	pr_debug("%s %s port %u mode %s\n", a.set[O_REMOVE] ? "Removing" : "Adding", protostr,
		 port, modestr);
	if (!(flags & (XFG_MAP_FLAG_DST | XFG_MAP_FLAG_SRC)) ||
	    !(flags & (XFG_MAP_FLAG_TCP | XFG_MAP_FLAG_UDP)))
		flags = 0;
	err = set_flags(ctx, XFG_MAP_PORTS, &key, flags, false);
	if (!err)
		err = xfg_store_save(ctx, state_dir);
	if (!err && a.set[O_STATUS])
		err = print_ports(ctx);
	xfg_close(ctx);
	lock_release(lock);
	return err ? 1 : 0;
}

static int do_address(int argc, char **argv, bool ether)
{
	static const struct opt opts[] = {
		{ "remove", 'r', false, O_REMOVE }, { "mode", 'm', true, O_MODE },
		{ "status", 's', false, O_STATUS }, { 0, 0, 0, 0 } };
	const char *usage = ether ?
		"Usage: xdp-filter ether [options] <addr>\n"
		"  -r, --remove              Remove address instead of adding\n"
		"  -m, --mode <mode>         Filter mode; default dst (valid values: src,dst)\n"
		"  -s, --status              Print status of filtered addresses after changing\n" :
		"Usage: xdp-filter ip [options] <addr>\n"
		"  -r, --remove              Remove address instead of adding\n"
		"  -m, --mode <mode>         Filter mode; default dst (valid values: src,dst)\n"
		"  -s, --status              Print status of filtered addresses after changing\n";
	struct args a;
	unsigned mode = XFG_MAP_FLAG_DST;
	uint8_t key[16];
	int map;
	int err = parse_args(argc, argv, opts, &a, usage);
	if (err)
		return err > 0 ? 0 : 1;
	if (a.npos != 1 || (a.set[O_MODE] && parse_flags(a.val[O_MODE], map_flags_srcdst, &mode))) {
		pr_warn("Invalid or missing parameter\n%s", usage);
		return 1;
	}
	const char *s = a.pos[0];
	if (ether) {
		/* parse_mac(): six %x fields, each <= 0xff (lib/util/params.c:147-165) */
		unsigned v[6];
		char extra;
		if (sscanf(s, "%x:%x:%x:%x:%x:%x%c", &v[0], &v[1], &v[2], &v[3], &v[4], &v[5],
			   &extra) != 6) {
			pr_warn("Invalid MAC address: %s\n", s);
			return 1;
		}
		for (int i = 0; i < 6; i++) {
			if (v[i] > 0xff) {
				pr_warn("Invalid MAC address: %s\n", s);
				return 1;
			}
			key[i] = (uint8_t)v[i];
		}
		map = XFG_MAP_ETHERNET;
	} else {
		/* handle_ipaddr(): a ':' means IPv6 (lib/util/params.c:308-322) */
		int af = strchr(s, ':') ? AF_INET6 : AF_INET;
		if (inet_pton(af, s, key) != 1) {
			pr_warn("Invalid IP address: %s\n", s);
			return 1;
		}
		map = af == AF_INET6 ? XFG_MAP_IPV6 : XFG_MAP_IPV4;
	}
	char modestr[100];
	print_flags(modestr, sizeof(modestr), map_flags_srcdst, mode);
	pr_debug("%s addr %s mode %s\n", a.set[O_REMOVE] ? "Removing" : "Adding", s, modestr);
	int lock = lock_acquire(false);
	if (lock < 0 || !xfg_store_has_map(state_dir, map)) {
		pr_warn("Couldn't find filter map; is xdp-filter loaded with the %s feature?\n",
			map == XFG_MAP_ETHERNET ? "ethernet" : map == XFG_MAP_IPV6 ? "ipv6" : "ipv4");
		lock_release(lock);
		return 1;
	}
	xfg_ctx *ctx = open_store(&err);
	if (!ctx) {
		lock_release(lock);
		return 1;
	}
	uint8_t flags = 0;
	uint64_t counter;
	get_counter_flags(ctx, map, key, &counter, &flags);
	if (a.set[O_REMOVE])
		flags &= ~mode;
	else
		flags |= mode;
	err = set_flags(ctx, map, key, flags, true);
	if (!err)
		err = xfg_store_save(ctx, state_dir);
	if (!err && a.set[O_STATUS])
		err = ether ? print_ethers(ctx) : print_ips(ctx);
	xfg_close(ctx);
	lock_release(lock);
	return err ? 1 : 0;
}

/* ------------------------------------------------------------------ status */
static int stats_print_one(const struct xfg_stats_record *st)
{
	/* lib/util/stats.c:48-71, ABORTED / DROP / PASS enabled (xdp-filter.c:981-983) */
	for (int i = 0; i < 3; i++)
		printf("  %-35s %'11lld pkts %'11lld KiB\n", action2str(i),
		       (long long)st[i].packets, (long long)(st[i].bytes / 1024));
	return 0;
}

static int do_status(int argc, char **argv)
{
	static const struct opt opts[] = { { 0, 0, 0, 0 } };
	struct args a;
	struct xfg_stats_record st[XFG_ACTION_MAX];
	int err = parse_args(argc, argv, opts, &a, "Usage: xdp-filter status\n");
	if (err)
		return err > 0 ? 0 : 1;
	int lock = lock_acquire(false);
	if (lock < 0 || xfg_store_stats_read(state_dir, st)) {
		pr_warn("Couldn't find stats map. Maybe xdp-filter is not loaded?\n");
		lock_release(lock);
		return 1;
	}
	xfg_ctx *ctx = open_store(&err);
	if (!ctx) {
		lock_release(lock);
		return 1;
	}
	printf("CURRENT XDP-FILTER STATUS:\n\n");
	printf("Aggregate per-action statistics:\n");
	stats_print_one(st);
	printf("\n");

	printf("Loaded on interfaces:\n");
	printf("  %-40s Enabled features\n", "");
	struct prog_rec *v;
	int n;
	if (!list_progs(&v, &n)) {
		for (int i = 0; i < n; i++) {
			char featbuf[100], namebuf[400];
			printf("%s\n", v[i].prog);
			print_flags(featbuf, sizeof(featbuf), print_features, find_features(v[i].prog));
			snprintf(namebuf, sizeof(namebuf), "%s (%s mode)", v[i].ifname, v[i].mode);
			printf("  %-40s %s\n", namebuf, featbuf);
		}
		free(v);
	}
	printf("\n");
	if (xfg_store_has_map(state_dir, XFG_MAP_PORTS)) {
		if ((err = print_ports(ctx)))
			goto out;
		printf("\n");
	}
	err = print_ips(ctx);
	if (err && err != -ENOENT)
		goto out;
	err = 0;
	printf("\n");
	if (xfg_store_has_map(state_dir, XFG_MAP_ETHERNET) && (err = print_ethers(ctx)))
		goto out;
	printf("\n");
out:
	xfg_close(ctx);
	lock_release(lock);
	return err ? 1 : 0;
}

/* ------------------------------------------------------------------ poll */
static volatile sig_atomic_t stop_poll;

static void on_signal(int sig)
{
	(void)sig;
	stop_poll = 1;
}

struct poll_rec {
	struct xfg_stats_record st[XFG_ACTION_MAX];
	uint64_t ts;
};

static uint64_t mono_ns(void)
{
	struct timespec t;
	clock_gettime(CLOCK_MONOTONIC, &t);
	return (uint64_t)t.tv_sec * 1000000000ull + t.tv_nsec;
}

/* stats_print() (lib/util/stats.c:73-125): DROP, PASS, TX, REDIRECT enabled */
static void stats_print(const struct poll_rec *r, const struct poll_rec *p)
{
	static const int enabled[] = { 1, 2, 3, 4 };
	double period = (r->ts - p->ts) / 1e9;
	struct timespec t;
	if (period <= 0)
		return;
	clock_gettime(CLOCK_REALTIME, &t);
	printf("Period of %fs ending at %ld.%06ld\n", period, (long)t.tv_sec,
	       (long)t.tv_nsec / 1000);
	for (int k = 0; k < 4; k++) {
		int i = enabled[k];
		uint64_t pk = r->st[i].packets - p->st[i].packets;
		uint64_t by = r->st[i].bytes - p->st[i].bytes;
		printf("%-12s %'11lld pkts (%'10.0f pps) %'11lld KiB (%'6.0f Mbits/s)\n",
		       action2str(i), (long long)r->st[i].packets, pk / period,
		       (long long)(r->st[i].bytes / 1024), by * 8 / period / 1000000);
	}
	printf("\n");
	fflush(stdout);
}

static int do_poll(int argc, char **argv)
{
	static const struct opt opts[] = {
		{ "interval", 'i', true, O_INTERVAL }, { "count", 'n', true, O_COUNT }, { 0, 0, 0, 0 } };
	const char *usage = "Usage: xdp-filter poll [options]\n"
			    "  -i, --interval <interval>  Polling interval in milliseconds (default 1000)\n"
			    "  -n, --count <n>            Stop after <n> reports (default: until interrupted)\n";
	struct args a;
	uint32_t interval = 1000, count = 0;
	int err = parse_args(argc, argv, opts, &a, usage);
	if (err)
		return err > 0 ? 0 : 1;
	if ((a.set[O_INTERVAL] && parse_u32(a.val[O_INTERVAL], 0xffffffffu, &interval)) ||
	    (a.set[O_COUNT] && parse_u32(a.val[O_COUNT], 0xffffffffu, &count))) {
		pr_warn("Invalid option value\n%s", usage);
		return 1;
	}
	if (!interval) {
		pr_warn("Can't use a polling interval of 0\n");
		return 1;
	}
	struct poll_rec rec, prev;
	if (xfg_store_stats_read(state_dir, rec.st)) {
		pr_warn("Couldn't find stats map. Maybe xdp-filter is not loaded?\n");
		return 1;
	}
	rec.ts = mono_ns();
	signal(SIGINT, on_signal);
	signal(SIGTERM, on_signal);
	usleep(1000000 / 4);
	for (uint32_t n = 0; !stop_poll && (!count || n < count); n++) {
		prev = rec;
		if (xfg_store_stats_read(state_dir, rec.st)) {
			pr_warn("Stats map disappeared while polling\n");
			pr_warn("Error polling statistics: %s\n", strerror(ENOENT));
			return 1;
		}
		rec.ts = mono_ns();
		stats_print(&rec, &prev);
		if (!count || n + 1 < count)
			usleep(interval * 1000);
	}
	return 0;
}

/* ------------------------------------------------------------------ run */
struct shard {
	xfg_ctx *ctx;
	int dev;
	struct xfg_batch b;
	uint8_t *verdicts;
	int repeat;
	int err;
};

static void *run_shard(void *arg)
{
	struct shard *s = arg;
	for (int r = 0; r < s->repeat && !s->err; r++)
		s->err = s->b.count ? xfg_classify_host(s->ctx, s->dev, &s->b, s->verdicts) : 0;
	return NULL;
}

static int do_run(int argc, char **argv)
{
	static const struct opt opts[] = {
		{ "gpus", 'g', true, O_GPUS }, { "dump", 'd', true, O_DUMP },
		{ "repeat", 'n', true, O_REPEAT }, { "quiet", 'q', false, O_QUIET }, { 0, 0, 0, 0 } };
	const char *usage =
		"Usage: xdp-filter run [options] <ifname> <capture>\n"
		"Classify a pcap/pcapng capture as traffic arriving on <ifname> with the program\n"
		"loaded there, on the GPUs; hit counters and statistics are updated in the store.\n"
		"  -g, --gpus <n>            GPUs to shard the capture over (default 1)\n"
		"  -d, --dump <file>         Write a pcapng with each packet's XDP verdict\n"
		"  -n, --repeat <k>          Classify the capture k times (default 1)\n"
		"  -q, --quiet               No summary line\n";
	struct args a;
	uint32_t ngpu = 1, repeat = 1;
	int err = parse_args(argc, argv, opts, &a, usage);
	if (err)
		return err > 0 ? 0 : 1;
	if (a.npos != 2 || (a.set[O_GPUS] && (parse_u32(a.val[O_GPUS], 64, &ngpu) || !ngpu)) ||
	    (a.set[O_REPEAT] && (parse_u32(a.val[O_REPEAT], 1u << 20, &repeat) || !repeat))) {
		pr_warn("Invalid or missing parameter\n%s", usage);
		return 1;
	}
	const char *ifname = a.pos[0], *capture = a.pos[1];
	int lock = lock_acquire(false);
	struct prog_rec r;
	if (lock < 0 || read_prog(ifname, &r)) {
		pr_warn("xdp-filter is not loaded on %s\n", ifname);
		lock_release(lock);
		return 1;
	}
	struct xfg_host_batch hb;
	if ((err = xfg_pcap_read(capture, &hb))) {
		pr_warn("Couldn't read capture %s: %s\n", capture, strerror(-err));
		lock_release(lock);
		return 1;
	}
	struct xfg_open_opts o;
	memset(&o, 0, sizeof(o));
	o.sz = sizeof(o);
	o.features = find_features(r.prog);
	o.ndev = (int)ngpu;
	int64_t c;
	if ((c = xfg_store_map_capacity(state_dir, XFG_MAP_IPV4)) > 0)
		o.ipv4_capacity = (uint32_t)c;
	if ((c = xfg_store_map_capacity(state_dir, XFG_MAP_IPV6)) > 0)
		o.ipv6_capacity = (uint32_t)c;
	if ((c = xfg_store_map_capacity(state_dir, XFG_MAP_ETHERNET)) > 0)
		o.eth_capacity = (uint32_t)c;
	xfg_ctx *ctx = NULL;
	uint8_t *verdicts = calloc(hb.count ? hb.count : 1, 1);
	struct shard *sh = calloc(ngpu, sizeof(*sh));
	pthread_t *th = calloc(ngpu, sizeof(*th));
	err = !verdicts || !sh || !th ? -ENOMEM : xfg_open(&ctx, &o);
	if (!err)
		err = xfg_store_load(ctx, state_dir);
	if (err) {
		pr_warn("Couldn't set up the classifier: %s\n", xfg_strerror(err));
		goto out;
	}
	pr_debug("Classifying %" PRIu64 " packets from %s with %s on %u GPU(s)\n", hb.count,
		 capture, xfg_prog_name(ctx), ngpu);
	uint64_t t0 = mono_ns();
	for (uint32_t d = 0; d < ngpu; d++) {
		uint64_t lo = hb.count * d / ngpu, hi = hb.count * (d + 1) / ngpu;
		sh[d] = (struct shard){ ctx, (int)d,
			{ hb.data, hb.offsets + lo, hb.lens + lo, hi - lo, 0, 0 },
			verdicts + lo, (int)repeat, 0 };
		if (pthread_create(&th[d], NULL, run_shard, &sh[d]))
			sh[d].err = -EAGAIN;
	}
	for (uint32_t d = 0; d < ngpu; d++) {
		if (sh[d].err != -EAGAIN)
			pthread_join(th[d], NULL);
		if (sh[d].err && !err)
			err = sh[d].err;
	}
	double secs = (mono_ns() - t0) / 1e9;
	if (err) {
		pr_warn("Classification failed: %s\n", xfg_strerror(err));
		goto out;
	}
	struct xfg_stats_record add[XFG_ACTION_MAX], st[XFG_ACTION_MAX];
	if ((err = xfg_stats_read(ctx, add)))
		goto out;
	if (xfg_store_stats_read(state_dir, st))
		memset(st, 0, sizeof(st));
	for (int i = 0; i < XFG_ACTION_MAX; i++) {
		st[i].packets += add[i].packets;
		st[i].bytes += add[i].bytes;
	}
	if ((err = xfg_store_save(ctx, state_dir)) || (err = xfg_store_stats_write(state_dir, st))) {
		pr_warn("Couldn't update the rule store: %s\n", strerror(-err));
		goto out;
	}
	if (a.set[O_DUMP] &&
	    (err = xfg_pcapng_write_verdicts(a.val[O_DUMP], ifname, &hb, verdicts))) {
		pr_warn("Couldn't write %s: %s\n", a.val[O_DUMP], strerror(-err));
		goto out;
	}
	if (!a.set[O_QUIET]) {
		uint64_t n = hb.count * (uint64_t)repeat;
		printf("Classified %" PRIu64 " packets on %s with %s (%u GPU(s)) in %.3f s: "
		       "%.1f Mpps incl. host<->GPU copies; %s %" PRIu64 " %s %" PRIu64 " %s %" PRIu64 "\n",
		       n, ifname, xfg_prog_name(ctx), ngpu, secs, secs > 0 ? n / secs / 1e6 : 0.0,
		       action2str(0), add[0].packets, action2str(1), add[1].packets, action2str(2),
		       add[2].packets);
	}
out:
	xfg_close(ctx);
	xfg_host_batch_free(&hb);
	free(verdicts);
	free(sh);
	free(th);
	lock_release(lock);
	return err ? 1 : 0;
}

/* ------------------------------------------------------------------ main */
static int do_help(void)
{
	fprintf(stderr,
		"Usage: xdp-filter COMMAND [options]\n"
		"\n"
		"COMMAND can be one of:\n"
		"       load        - load xdp-filter on an interface\n"
		"       unload      - unload xdp-filter from an interface\n"
		"       port        - add a port to the filter list\n"
		"       ip          - add an IP address to the filter list\n"
		"       ether       - add an Ethernet MAC address to the filter list\n"
		"       status      - show current xdp-filter status\n"
		"       poll        - poll statistics output\n"
		"       run         - classify a capture on the GPUs (MI355X)\n"
		"       help        - show this help message\n"
		"\n"
		"Use 'xdp-filter COMMAND --help' to see options for each command\n");
	return -1;
}

int main(int argc, char **argv)
{
	init_state_dir();
	if (argc < 2)
		return do_help() ? 1 : 0;
	const char *cmd = argv[1];
	argc--;
	argv++;
	if (!strcmp(cmd, "load"))
		return do_load(argc, argv);
	if (!strcmp(cmd, "unload"))
		return do_unload(argc, argv);
	if (!strcmp(cmd, "port"))
		return do_port(argc, argv);
	if (!strcmp(cmd, "ip"))
		return do_address(argc, argv, false);
	if (!strcmp(cmd, "ether"))
		return do_address(argc, argv, true);
	if (!strcmp(cmd, "status"))
		return do_status(argc, argv);
	if (!strcmp(cmd, "poll"))
		return do_poll(argc, argv);
	if (!strcmp(cmd, "run"))
		return do_run(argc, argv);
	if (!strcmp(cmd, "help"))
		return do_help() ? 1 : 0;
	fprintf(stderr, "Command '%s' is unknown, try '%s help'.\n", cmd, PROG_NAME);
	return 1;
}
