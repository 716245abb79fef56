// The drop-in as DuckDB would load it: a C++ caller that declares the backend
// symbols the way the reference's src/rust_ffi.cpp:7-42 expects them (same
// names, same parameter types, extern "C", separate translation unit, no
// include of lancedb_hip.h), links liblancedb_hip.so, and never loads torch —
// so the library runs on the HIP runtime it was linked against (/opt/rocm),
// exactly what the link swap of CMakeLists.txt:117-121 gives a DuckDB process.
//
//   abi_caller                 null-handle / error-buffer checks (no GPU needed)
//   abi_caller gpu SCRIPT      runs SCRIPT (see run_script) against the device
//
// The GPU mode restates the two C++ layers above the C-ABI with the
// reference's semantics: RustFFI (rust_ffi.cpp:44-208: 2048-byte err_buf,
// IOException "Lance <op>: msg" on a NULL / negative return) and MiniIndex
// (lance_index.cpp: lazy dataset creation on the first Append :283-312,
// label_to_rowid_ / rowid_to_label_ :949-954, Delete :389-425, Search's
// dimension guard and label -> row id mapping :442-465, CHECKPOINT + restart
// as Serialize / LoadFromStorage :492-587).  Multi-column rows go through the
// Arrow C Data Interface as DuckDB's ArrowConverter hands them over
// (lance_index.cpp:322-360).
#include <algorithm>
#include <cerrno>
#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <map>
#include <memory>
#include <set>
#include <sstream>
#include <stdexcept>
#include <string>
#include <vector>

extern "C" {
void *lance_create_detached(const char *, int32_t, const char *, const char *, char *, int);
void *lance_create_detached_from_arrow(const char *, void *, const char *, const char *, char *, int);
void *lance_open_detached(const char *, const char *, const char *, char *, int);
void lance_free_detached(void *);
int32_t lance_detached_has_extra_columns(void *);
int32_t lance_detached_dimension(void *);
int64_t lance_detached_add(void *, const float *, int32_t, char *, int);
int32_t lance_detached_add_batch(void *, const float *, int32_t, int32_t, int64_t *, char *, int);
int32_t lance_detached_add_batch_arrow(void *, void *, void *, int64_t *, char *, int);
int32_t lance_detached_merge(void *, void *, const int64_t *, int32_t, int64_t *, int64_t *, char *, int);
int32_t lance_detached_search(void *, const float *, int32_t, int32_t, int32_t, int32_t, int64_t *, float *, char *,
                              int);
int64_t lance_detached_count(void *, char *, int);
int32_t lance_detached_delete(void *, int64_t, char *, int);
int32_t lance_detached_delete_batch(void *, const int64_t *, int32_t, char *, int);
int32_t lance_detached_create_index(void *, int32_t, int32_t, char *, int);
int32_t lance_detached_create_hnsw_index(void *, int32_t, int32_t, char *, int);
int32_t lance_detached_compact(void *, char *, int);
int32_t lance_detached_get_vector(void *, int64_t, float *, int32_t, char *, int);
int32_t lance_detached_get_all_vectors(void *, int64_t *, float *, int64_t *, char *, int);
// the intended predicate form (lance_index.cpp:452-453)
int32_t lance_detached_search_with_predicate(void *, const float *, int32_t, int32_t, int32_t, int32_t, const char *,
                                             int64_t *, float *, char *, int);
// the batched form
int32_t lance_detached_search_batch(void *, const float *, int32_t, int32_t, int32_t, int32_t, int32_t, const char *,
                                    int64_t *, float *, int32_t *, char *, int);
}

static int fails = 0;
static void expect(bool ok, const char *what) {
	if (!ok) {
		std::printf("FAIL %s\n", what);
		++fails;
	}
}

static int null_checks() {
	char err[2048];
	float q[3] = {1, 0, 0};
	int64_t labels[4];
	float dists[4];
	err[0] = 0;
	expect(lance_detached_search(nullptr, q, 3, 4, 20, 1, labels, dists, err, sizeof err) == -1, "search rc");
	expect(std::strcmp(err, "null handle") == 0, "search msg");
	expect(lance_detached_search_with_predicate(nullptr, q, 3, 4, 20, 1, "x = 1", labels, dists, err, sizeof err) ==
	           -1,
	       "pred rc");
	expect(lance_detached_count(nullptr, err, sizeof err) == -1, "count");
	expect(lance_detached_add(nullptr, q, 3, err, sizeof err) == -1, "add");
	expect(lance_detached_add_batch(nullptr, q, 1, 3, labels, err, sizeof err) == -1, "add_batch");
	expect(lance_detached_delete(nullptr, 0, err, sizeof err) == -1, "delete");
	expect(lance_detached_delete_batch(nullptr, labels, 1, err, sizeof err) == -1, "delete_batch");
	expect(lance_detached_create_index(nullptr, 4, 2, err, sizeof err) == -1, "create_index");
	expect(lance_detached_create_hnsw_index(nullptr, 4, 2, err, sizeof err) == -1, "create_hnsw");
	expect(lance_detached_compact(nullptr, err, sizeof err) == -1, "compact");
	expect(lance_detached_get_vector(nullptr, 0, dists, 4, err, sizeof err) == -1, "get_vector");
	expect(lance_detached_get_all_vectors(nullptr, nullptr, nullptr, nullptr, err, sizeof err) == -1, "get_all");
	expect(lance_detached_merge(nullptr, nullptr, labels, 1, labels, labels, err, sizeof err) == -1, "merge");
	expect(lance_detached_add_batch_arrow(nullptr, nullptr, nullptr, labels, err, sizeof err) == -1, "arrow add");
	expect(lance_create_detached_from_arrow("", nullptr, "l2", "t", err, sizeof err) == nullptr, "arrow create");
	expect(lance_detached_dimension(nullptr) == 0, "dimension");
	expect(lance_detached_has_extra_columns(nullptr) == 0, "extra cols");
	lance_free_detached(nullptr);
	(void)lance_create_detached;
	(void)lance_open_detached;
	std::printf(fails ? "FAILED\n" : "OK\n");
	return fails ? 1 : 0;
}

// ---------------------------------------------------------------------------
// rust_ffi.cpp restated: one wrapper per symbol, 2048-byte err_buf, throws
// ---------------------------------------------------------------------------
struct IOException : std::runtime_error {
	using std::runtime_error::runtime_error;
};

namespace RustFFI {
static constexpr int ERR_LEN = 2048;  // rust_ffi.cpp:46
static void *CreateDetached(const std::string &path, int dim, const std::string &metric, const std::string &table) {
	char e[ERR_LEN] = {0};
	void *h = lance_create_detached(path.c_str(), dim, metric.c_str(), table.c_str(), e, ERR_LEN);
	if (!h) throw IOException(std::string("Lance create: ") + e);
	return h;
}
static void *CreateFromArrow(const std::string &path, void *schema, const std::string &metric,
                             const std::string &table) {
	char e[ERR_LEN] = {0};
	void *h = lance_create_detached_from_arrow(path.c_str(), schema, metric.c_str(), table.c_str(), e, ERR_LEN);
	if (!h) throw IOException(std::string("Lance create_from_arrow: ") + e);
	return h;
}
static void *OpenDetached(const std::string &path, const std::string &table, const std::string &metric) {
	char e[ERR_LEN] = {0};
	void *h = lance_open_detached(path.c_str(), table.c_str(), metric.c_str(), e, ERR_LEN);
	if (!h) throw IOException(std::string("Lance open: ") + e);
	return h;
}
static int64_t Add(void *h, const float *v, int dim) {
	char e[ERR_LEN] = {0};
	int64_t l = lance_detached_add(h, v, dim, e, ERR_LEN);
	if (l < 0) throw IOException(std::string("Lance add: ") + e);
	return l;
}
static void AddBatch(void *h, const float *v, int num, int dim, int64_t *out) {
	char e[ERR_LEN] = {0};
	if (lance_detached_add_batch(h, v, num, dim, out, e, ERR_LEN) < 0)
		throw IOException(std::string("Lance add_batch: ") + e);
}
static int AddBatchArrow(void *h, void *schema, void *array, int64_t *out) {
	char e[ERR_LEN] = {0};
	int n = lance_detached_add_batch_arrow(h, schema, array, out, e, ERR_LEN);
	if (n < 0) throw IOException(std::string("Lance add_batch_arrow: ") + e);
	return n;
}
static int Search(void *h, const float *q, int dim, int k, int nprobes, int refine, const char *pred, int64_t *labels,
                  float *dists) {
	char e[ERR_LEN] = {0};
	int n = pred ? lance_detached_search_with_predicate(h, q, dim, k, nprobes, refine, pred, labels, dists, e, ERR_LEN)
	             : lance_detached_search(h, q, dim, k, nprobes, refine, labels, dists, e, ERR_LEN);
	if (n < 0) throw IOException(std::string("Lance search: ") + e);
	return n;
}
static void SearchBatch(void *h, const float *Q, int nq, int dim, int k, const char *pred, int64_t *labels,
                        float *dists, int32_t *counts) {
	char e[ERR_LEN] = {0};
	if (lance_detached_search_batch(h, Q, nq, dim, k, 20, 1, pred, labels, dists, counts, e, ERR_LEN) < 0)
		throw IOException(std::string("Lance search: ") + e);
}
static int64_t Count(void *h) {
	char e[ERR_LEN] = {0};
	int64_t n = lance_detached_count(h, e, ERR_LEN);
	if (n < 0) throw IOException(std::string("Lance count: ") + e);
	return n;
}
static void DeleteBatch(void *h, const int64_t *labels, int n) {
	char e[ERR_LEN] = {0};
	if (lance_detached_delete_batch(h, labels, n, e, ERR_LEN) != 0)
		throw IOException(std::string("Lance delete_batch: ") + e);
}
static void Delete(void *h, int64_t label) {
	char e[ERR_LEN] = {0};
	if (lance_detached_delete(h, label, e, ERR_LEN) != 0) throw IOException(std::string("Lance delete: ") + e);
}
static void CreateHnsw(void *h, int m, int ef) {
	char e[ERR_LEN] = {0};
	if (lance_detached_create_hnsw_index(h, m, ef, e, ERR_LEN) != 0)
		throw IOException(std::string("Lance create_hnsw_index: ") + e);
}
}  // namespace RustFFI

// ---------------------------------------------------------------------------
// Arrow C Data Interface: a struct batch [vector FixedSizeList<f32>[d], lang
// utf8 (nullable), score int32], everything owned by the root's private data
// ---------------------------------------------------------------------------
struct ArrowSchema {
	const char *format, *name, *metadata;
	int64_t flags, n_children;
	ArrowSchema **children;
	ArrowSchema *dictionary;
	void (*release)(ArrowSchema *);
	void *private_data;
};
struct ArrowArray {
	int64_t length, null_count, offset, n_buffers, n_children;
	const void **buffers;
	ArrowArray **children;
	ArrowArray *dictionary;
	void (*release)(ArrowArray *);
	void *private_data;
};

struct DocBatch {  // backing store of one exported batch
	ArrowSchema s_root{}, s_vec{}, s_val{}, s_lang{}, s_score{};
	ArrowArray a_root{}, a_vec{}, a_val{}, a_lang{}, a_score{};
	ArrowSchema *s_kids[3], *s_veckid[1];
	ArrowArray *a_kids[3], *a_veckid[1];
	const void *b_root[1], *b_vec[1], *b_val[2], *b_lang[3], *b_score[2];
	std::string vec_fmt;
	std::vector<float> vals;
	std::vector<int32_t> offs, scores;
	std::string chars;
	std::vector<uint8_t> lang_valid, score_valid;
};

static void release_child_schema(ArrowSchema *s) { s->release = nullptr; }
static void release_child_array(ArrowArray *a) { a->release = nullptr; }
static void release_root_schema(ArrowSchema *s) {
	for (int i = 0; i < 3; ++i)
		if (s->children[i]->release) s->children[i]->release(s->children[i]);
	s->release = nullptr;
}
static void release_root_array(ArrowArray *a) {
	for (int i = 0; i < 3; ++i)
		if (a->children[i]->release) a->children[i]->release(a->children[i]);
	a->release = nullptr;
}

// lang[i] empty string with lang_null[i] = NULL; score likewise
static std::unique_ptr<DocBatch> make_doc_batch(const std::vector<float> &rows, int n, int d,
                                                const std::vector<std::string> &lang, const std::vector<char> &lang_null,
                                                const std::vector<int32_t> &score, const std::vector<char> &score_null) {
	auto b = std::make_unique<DocBatch>();
	b->vals = rows;
	b->vec_fmt = "+w:" + std::to_string(d);
	b->offs.assign((size_t)n + 1, 0);
	b->lang_valid.assign((size_t)(n + 7) / 8, 0);
	b->score_valid.assign((size_t)(n + 7) / 8, 0);
	b->scores = score;
	int64_t lnull = 0, snull = 0;
	for (int i = 0; i < n; ++i) {
		if (!lang_null[(size_t)i]) {
			b->chars += lang[(size_t)i];
			b->lang_valid[(size_t)i / 8] |= (uint8_t)(1u << (i % 8));
		} else {
			++lnull;
		}
		b->offs[(size_t)i + 1] = (int32_t)b->chars.size();
		if (!score_null[(size_t)i])
			b->score_valid[(size_t)i / 8] |= (uint8_t)(1u << (i % 8));
		else
			++snull;
	}
	auto sch = [](ArrowSchema &s, const char *fmt, const char *name, int64_t nk, ArrowSchema **kids, bool root) {
		s.format = fmt;
		s.name = name;
		s.metadata = nullptr;
		s.flags = 2;  // ARROW_FLAG_NULLABLE
		s.n_children = nk;
		s.children = kids;
		s.dictionary = nullptr;
		s.release = root ? release_root_schema : release_child_schema;
		s.private_data = nullptr;
	};
	b->s_veckid[0] = &b->s_val;
	b->s_kids[0] = &b->s_vec;
	b->s_kids[1] = &b->s_lang;
	b->s_kids[2] = &b->s_score;
	sch(b->s_root, "+s", "", 3, b->s_kids, true);
	sch(b->s_vec, b->vec_fmt.c_str(), "embedding", 1, b->s_veckid, false);
	sch(b->s_val, "f", "item", 0, nullptr, false);
	sch(b->s_lang, "u", "lang", 0, nullptr, false);
	sch(b->s_score, "i", "score", 0, nullptr, false);
	auto arr = [](ArrowArray &a, int64_t len, int64_t nulls, int64_t nb, const void **bufs, int64_t nk,
	              ArrowArray **kids, bool root) {
		a.length = len;
		a.null_count = nulls;
		a.offset = 0;
		a.n_buffers = nb;
		a.n_children = nk;
		a.buffers = bufs;
		a.children = kids;
		a.dictionary = nullptr;
		a.release = root ? release_root_array : release_child_array;
		a.private_data = nullptr;
	};
	b->b_root[0] = nullptr;
	b->b_vec[0] = nullptr;
	b->b_val[0] = nullptr;
	b->b_val[1] = b->vals.data();
	b->b_lang[0] = b->lang_valid.data();
	b->b_lang[1] = b->offs.data();
	b->b_lang[2] = b->chars.data();
	b->b_score[0] = b->score_valid.data();
	b->b_score[1] = b->scores.data();
	b->a_veckid[0] = &b->a_val;
	b->a_kids[0] = &b->a_vec;
	b->a_kids[1] = &b->a_lang;
	b->a_kids[2] = &b->a_score;
	arr(b->a_root, n, 0, 1, b->b_root, 3, b->a_kids, true);
	arr(b->a_vec, n, 0, 1, b->b_vec, 1, b->a_veckid, false);
	arr(b->a_val, (int64_t)n * d, 0, 2, b->b_val, 0, nullptr, false);
	arr(b->a_lang, n, lnull, 3, b->b_lang, 0, nullptr, false);
	arr(b->a_score, n, snull, 2, b->b_score, 0, nullptr, false);
	return b;
}

// ---------------------------------------------------------------------------
// lance_index.cpp restated (the hot-path subset DuckDB drives)
// ---------------------------------------------------------------------------
struct MiniIndex {
	int dim;
	std::string metric, path, table;
	bool with_cols;
	int nprobes = 20, refine_factor = 1;  // lance_index.hpp:91-92
	void *handle = nullptr;
	std::vector<int64_t> label_to_rowid;
	std::map<int64_t, int64_t> rowid_to_label;

	MiniIndex(int d, std::string m, std::string p, std::string t, bool cols)
	    : dim(d), metric(std::move(m)), path(std::move(p)), table(std::move(t)), with_cols(cols) {}
	~MiniIndex() {
		if (handle) lance_free_detached(handle);  // CommitDrop (lance_index.cpp:427-436)
	}
	void record(const int64_t *labels, int n, const int64_t *rowids) {
		for (int i = 0; i < n; ++i) {
			if ((int64_t)label_to_rowid.size() <= labels[i]) label_to_rowid.resize((size_t)labels[i] + 1, -1);
			label_to_rowid[(size_t)labels[i]] = rowids[i];
			rowid_to_label[rowids[i]] = labels[i];
		}
	}
	// Append (lance_index.cpp:273-383), vector-only fast path: the FLOAT[N]
	// child buffer straight to add_batch (:940-946)
	void Append(const float *rows, int n, const int64_t *rowids) {
		if (n == 0) return;
		if (!handle) handle = RustFFI::CreateDetached(path, dim, metric, table);
		std::vector<int64_t> labels((size_t)n);
		RustFFI::AddBatch(handle, rows, n, dim, labels.data());
		record(labels.data(), n, rowids);
	}
	// Append of a multi-column chunk through the Arrow C Data Interface (:322-360)
	void AppendCols(DocBatch &b, int n, const int64_t *rowids) {
		if (!handle) handle = RustFFI::CreateFromArrow(path, &b.s_root, metric, table);
		std::vector<int64_t> labels((size_t)n);
		const int got = RustFFI::AddBatchArrow(handle, &b.s_root, &b.a_root, labels.data());
		if (b.a_root.release) throw IOException("the callee did not take the Arrow array over");
		if (got != n) throw IOException("add_batch_arrow returned " + std::to_string(got));
		record(labels.data(), n, rowids);
	}
	// Delete (:389-425)
	void Delete(const int64_t *rowids, int n) {
		std::vector<int64_t> labels;
		for (int i = 0; i < n; ++i) {
			auto it = rowid_to_label.find(rowids[i]);
			if (it == rowid_to_label.end()) continue;
			labels.push_back(it->second);
			if (it->second >= 0 && it->second < (int64_t)label_to_rowid.size()) label_to_rowid[(size_t)it->second] = -1;
			rowid_to_label.erase(it);
		}
		if (handle && !labels.empty()) RustFFI::DeleteBatch(handle, labels.data(), (int)labels.size());
	}
	// Search (:442-465): {} on a dimension mismatch, labels -> row ids, labels
	// outside [0, size) dropped
	std::vector<std::pair<int64_t, float>> Search(const float *q, int qdim, int k, const std::string &pred) {
		std::vector<std::pair<int64_t, float>> out;
		if (!handle || qdim != dim || k <= 0) return out;
		std::vector<int64_t> labels((size_t)k);
		std::vector<float> dists((size_t)k);
		const int n = RustFFI::Search(handle, q, qdim, k, nprobes, refine_factor, pred.empty() ? nullptr : pred.c_str(),
		                              labels.data(), dists.data());
		for (int i = 0; i < n; ++i)
			if (labels[(size_t)i] >= 0 && labels[(size_t)i] < (int64_t)label_to_rowid.size())
				out.emplace_back(label_to_rowid[(size_t)labels[(size_t)i]], dists[(size_t)i]);
		return out;
	}
	// CHECKPOINT + restart: the metadata survives in DuckDB's index blocks
	// (PersistToDisk :492-532), the vectors are reopened (LoadFromStorage :534-587)
	void Restart() {
		if (handle) lance_free_detached(handle);
		handle = RustFFI::OpenDetached(path, table, metric);
	}
	int64_t Count() { return handle ? RustFFI::Count(handle) : 0; }
};

// ---------------------------------------------------------------------------
// script
// ---------------------------------------------------------------------------
static std::vector<char> read_file(const std::string &p, size_t want) {
	std::ifstream f(p, std::ios::binary);
	if (!f) throw std::runtime_error("cannot open " + p);
	std::vector<char> b(want);
	f.read(b.data(), (std::streamsize)want);
	if ((size_t)f.gcount() != want) throw std::runtime_error("short read " + p);
	return b;
}
static void write_file(const std::string &p, const void *d, size_t n, bool append) {
	FILE *f = std::fopen(p.c_str(), append ? "ab" : "wb");
	if (!f) throw std::runtime_error("cannot write " + p);
	std::fwrite(d, 1, n, f);
	std::fclose(f);
}

// which HIP / HSA runtime and whether any torch library is mapped
static void print_maps() {
	std::ifstream f("/proc/self/maps");
	std::set<std::string> libs;
	bool torch = false;
	for (std::string line; std::getline(f, line);) {
		const size_t sp = line.find('/');
		if (sp == std::string::npos) continue;
		const std::string path = line.substr(sp);
		if (path.find("libamdhip64") != std::string::npos || path.find("libhsa-runtime64") != std::string::npos ||
		    path.find("liblancedb_hip") != std::string::npos)
			libs.insert(path);
		if (path.find("libtorch") != std::string::npos || path.find("libc10") != std::string::npos) torch = true;
	}
	for (const auto &l : libs) std::printf("maps %s\n", l.c_str());
	std::printf("torch %d\n", torch ? 1 : 0);
}

static std::string tok_or(std::istringstream &is, const char *dflt) {
	std::string t;
	if (!(is >> t)) return dflt;
	return t == "-" ? std::string() : t;
}

// Commands, one per line (floats in decimal, a '|' starts a trailing predicate):
//   maps
//   index DIM METRIC PATH TABLE [cols]      new MiniIndex ('-' = empty path)
//   append N ROWID*N FLOAT*(N*DIM)
//   append_cols N ROWID*N FLOAT*(N*DIM) LANG*N SCORE*N   ('\N' = NULL)
//   delete N ROWID*N
//   search K QDIM FLOAT*QDIM [| PRED]       -> "res n rowid dist ..."
//   count                                   -> "count n"
//   restart | hnsw M EF
//   raw_create SLOT DIM PATH TABLE | raw_open SLOT PATH TABLE | raw_free SLOT
//   raw_add SLOT DIM FLOAT*DIM -> "label l" | raw_delete SLOT LABEL | raw_count SLOT -> "count n"
//   bulk DIM METRIC BASE.bin N CHUNK        MiniIndex over BASE (f32 N x DIM), 2048-row Sink chunks
//   bulk_delete FILE.bin N                  rowids (int64)
//   bulk_search QFILE NQ K OUT percall|batch [| PRED]
//       OUT: rowids int64 [NQ][K] (-1 pad), dists f32 [NQ][K] (NaN pad), counts int32 [NQ]
static int run_script(const char *path) {
	std::ifstream f(path);
	if (!f) {
		std::printf("cannot open script %s\n", path);
		return 2;
	}
	std::unique_ptr<MiniIndex> ix;
	std::map<std::string, void *> raw;
	std::vector<float> bulk_rows;
	int lineno = 0;
	for (std::string line; std::getline(f, line);) {
		++lineno;
		std::string pred;
		const size_t bar = line.find('|');
		if (bar != std::string::npos) {
			pred = line.substr(bar + 1);
			while (!pred.empty() && pred[0] == ' ') pred.erase(0, 1);
			line = line.substr(0, bar);
		}
		std::istringstream is(line);
		std::string op;
		if (!(is >> op) || op[0] == '#') continue;
		try {
			if (op == "maps") {
				print_maps();
			} else if (op == "index") {
				int d;
				std::string m;
				is >> d >> m;
				const std::string p = tok_or(is, ""), t = tok_or(is, "vectors");
				std::string c;
				is >> c;
				ix = std::make_unique<MiniIndex>(d, m, p, t, c == "cols");
			} else if (op == "append" || op == "append_cols") {
				int n;
				is >> n;
				std::vector<int64_t> rid((size_t)n);
				for (auto &r : rid) is >> r;
				std::vector<float> rows((size_t)n * ix->dim);
				for (auto &v : rows) is >> v;
				if (op == "append") {
					ix->Append(rows.data(), n, rid.data());
				} else {
					std::vector<std::string> lang((size_t)n);
					std::vector<char> ln((size_t)n), sn((size_t)n);
					std::vector<int32_t> sc((size_t)n);
					for (int i = 0; i < n; ++i) {
						is >> lang[(size_t)i];
						ln[(size_t)i] = lang[(size_t)i] == "\\N";
					}
					for (int i = 0; i < n; ++i) {
						std::string s;
						is >> s;
						sn[(size_t)i] = s == "\\N";
						sc[(size_t)i] = sn[(size_t)i] ? 0 : std::atoi(s.c_str());
					}
					auto b = make_doc_batch(rows, n, ix->dim, lang, ln, sc, sn);
					ix->AppendCols(*b, n, rid.data());
					if (b->s_root.release) b->s_root.release(&b->s_root);  // the schema stays the caller's
				}
				if (!is) throw std::runtime_error("malformed append");
			} else if (op == "delete") {
				int n;
				is >> n;
				std::vector<int64_t> rid((size_t)n);
				for (auto &r : rid) is >> r;
				ix->Delete(rid.data(), n);
			} else if (op == "search") {
				int k, qd;
				is >> k >> qd;
				std::vector<float> q((size_t)qd);
				for (auto &v : q) is >> v;
				auto res = ix->Search(q.data(), qd, k, pred);
				std::printf("res %zu", res.size());
				for (auto &r : res) std::printf(" %lld %.9g", (long long)r.first, (double)r.second);
				std::printf("\n");
			} else if (op == "count") {
				std::printf("count %lld\n", (long long)ix->Count());
			} else if (op == "restart") {
				ix->Restart();
			} else if (op == "hnsw") {
				int m, ef;
				is >> m >> ef;
				RustFFI::CreateHnsw(ix->handle, m, ef);
			} else if (op == "raw_create") {
				std::string s;
				int d;
				is >> s >> d;
				const std::string p = tok_or(is, ""), t = tok_or(is, "vectors");
				raw[s] = RustFFI::CreateDetached(p, d, "l2", t);
			} else if (op == "raw_open") {
				std::string s;
				is >> s;
				const std::string p = tok_or(is, ""), t = tok_or(is, "vectors");
				raw[s] = RustFFI::OpenDetached(p, t, "l2");
			} else if (op == "raw_free") {
				std::string s;
				is >> s;
				lance_free_detached(raw[s]);
				raw.erase(s);
			} else if (op == "raw_add") {
				std::string s;
				int d;
				is >> s >> d;
				std::vector<float> v((size_t)d);
				for (auto &x : v) is >> x;
				std::printf("label %lld\n", (long long)RustFFI::Add(raw.at(s), v.data(), d));
			} else if (op == "raw_delete") {
				std::string s;
				long long l;
				is >> s >> l;
				RustFFI::Delete(raw.at(s), l);
			} else if (op == "raw_count") {
				std::string s;
				is >> s;
				std::printf("count %lld\n", (long long)RustFFI::Count(raw.at(s)));
			} else if (op == "bulk") {
				int d, chunk;
				long long n;
				std::string m, file;
				is >> d >> m >> file >> n >> chunk;
				auto b = read_file(file, (size_t)n * d * sizeof(float));
				ix = std::make_unique<MiniIndex>(d, m, "", "vectors", false);
				const float *rows = reinterpret_cast<const float *>(b.data());
				std::vector<int64_t> rid((size_t)chunk);
				for (long long s = 0; s < n; s += chunk) {
					const int c = (int)std::min<long long>(chunk, n - s);
					for (int i = 0; i < c; ++i) rid[(size_t)i] = s + i;
					ix->Append(rows + (size_t)s * d, c, rid.data());
				}
			} else if (op == "bulk_delete") {
				std::string file;
				int n;
				is >> file >> n;
				auto b = read_file(file, (size_t)n * sizeof(int64_t));
				ix->Delete(reinterpret_cast<const int64_t *>(b.data()), n);
			} else if (op == "bulk_search") {
				std::string qf, out, mode;
				int nq, k;
				is >> qf >> nq >> k >> out >> mode;
				const int d = ix->dim;
				auto b = read_file(qf, (size_t)nq * d * sizeof(float));
				const float *Q = reinterpret_cast<const float *>(b.data());
				std::vector<int64_t> L((size_t)nq * k, -1);
				std::vector<float> D((size_t)nq * k, NAN);
				std::vector<int32_t> C((size_t)nq, 0);
				if (mode == "percall") {
					// lance_search()'s pattern: one Search per query (lance_search.cpp:73-74)
					for (int i = 0; i < nq; ++i) {
						auto res = ix->Search(Q + (size_t)i * d, d, k, pred);
						C[(size_t)i] = (int32_t)res.size();
						for (size_t j = 0; j < res.size(); ++j) {
							L[(size_t)i * k + j] = res[j].first;
							D[(size_t)i * k + j] = res[j].second;
						}
					}
				} else {
					RustFFI::SearchBatch(ix->handle, Q, nq, d, k, pred.empty() ? nullptr : pred.c_str(), L.data(),
					                     D.data(), C.data());
					for (size_t i = 0; i < L.size(); ++i)  // labels -> row ids (bulk: the identity until deletes)
						if (L[i] >= 0) L[i] = ix->label_to_rowid.at((size_t)L[i]);
				}
				write_file(out, L.data(), L.size() * 8, false);
				write_file(out, D.data(), D.size() * 4, true);
				write_file(out, C.data(), C.size() * 4, true);
				std::printf("bulk_search %d\n", nq);
			} else if (op == "time_percall") {
				// lance_search()'s one-Search-per-query pattern timed from C++ (no
				// Python in the loop): `settle` untimed calls (the GPU clock ramp),
				// then `reps` passes over the nq queries
				std::string qf;
				int nq, k, settle, reps;
				is >> qf >> nq >> k >> settle >> reps;
				const int d = ix->dim;
				auto b = read_file(qf, (size_t)nq * d * sizeof(float));
				const float *Q = reinterpret_cast<const float *>(b.data());
				size_t got = 0;
				for (int i = 0; i < settle; ++i) got += ix->Search(Q + (size_t)(i % nq) * d, d, k, pred).size();
				std::vector<double> per;
				per.reserve((size_t)nq * reps);
				const auto t0 = std::chrono::steady_clock::now();
				auto tp = t0;
				for (int r = 0; r < reps; ++r)
					for (int i = 0; i < nq; ++i) {
						got += ix->Search(Q + (size_t)i * d, d, k, pred).size();
						const auto tn = std::chrono::steady_clock::now();
						per.push_back(std::chrono::duration<double, std::micro>(tn - tp).count());
						tp = tn;
					}
				const double s = std::chrono::duration<double>(tp - t0).count();
				std::sort(per.begin(), per.end());
				std::printf("time_percall %zu %.6f %.3f %.3f %zu\n", per.size(), s, 1e6 * s / (double)per.size(),
				            per[per.size() / 2], got);
			} else {
				throw std::runtime_error("unknown op " + op);
			}
		} catch (const std::exception &e) {
			std::printf("error %d %s\n", lineno, e.what());
		}
		std::fflush(stdout);
	}
	for (auto &kv : raw) lance_free_detached(kv.second);
	std::printf("done\n");
	return 0;
}

int main(int argc, char **argv) {
	if (argc >= 3 && std::strcmp(argv[1], "gpu") == 0) return run_script(argv[2]);
	return null_checks();
}
