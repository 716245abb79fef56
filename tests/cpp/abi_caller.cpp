// Link-compatibility check: a C++ caller that declares the backend symbols the
// way the reference's src/rust_ffi.cpp:7-42 expects them (same names, same
// parameter types, extern "C", separate translation unit, no include of
// lancedb_hip.h) and links against liblancedb_hip.so.  Exercises only paths
// that need no GPU (null handles, error buffers), so it runs on CPU hosts.
#include <cstdint>
#include <cstdio>
#include <cstring>

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
}

static int fails = 0;
static void expect(bool ok, const char *what) {
	if (!ok) {
		std::printf("FAIL %s\n", what);
		++fails;
	}
}

int main() {
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
