/*
 * TEST INFRASTRUCTURE ONLY -- never linked into libbcp.
 *
 * `make ref` compiles this file in ONE translation unit right after the
 * reference's own planner text, streamed unchanged from /root/reference by
 * ref_stream.sh (SHA-checked, no copy written):
 *
 *   common/common.h:15-34, 50-51     FileInfo, TEST_BIT/GET_P/WITH_P/NO_P, MAX
 *   gen/file_info_hash.h:12-16       FatFileInfo
 *   gen/assign_lanes.h:6-7           u64, assign_lanes()
 *   gen/main.c:52                    st_weight[]
 *   gen/main.c:60-74                 sts_in_use, simple_hash
 *   gen/main.c:92-100                fill_in_missing_fields
 *   gen/main.c:174-189               SizeIndex, cmp_entries
 *   gen/main.c:338-401               PCG32, shuffle, select_P
 *   gen/main.c:403-427               get_store_weight
 *   gen/file_info_hash.c:24-31       fih_add_info
 *   gen/assign_lanes.c:7-46          assign_lanes
 *
 * and exports them as ref_* for tests/golden/make_ref_plan_golden.py and the
 * CPU tests.  The pieces below that are glue of mine are a few lines each
 * that sequence reference functions exactly as the reference's caller does
 * (the caller itself needs MPI / LevelDB and is not compiled): ref_sort_order
 * (gen/main.c:710-711), ref_round_order[_ranked] (:310, :710-711, :758) and
 * ref_plan_item (gen/main.c:772-788 around pdb_get).
 * Output: oracle/_ref/libref_plan.so (git-ignored).
 */

unsigned ref_simple_hash(const char *p, int len)
{
    return simple_hash(p, len);
}

int ref_sts_in_use(uint64_t locations)
{
    return sts_in_use(locations);
}

void ref_pcg32(uint64_t initstate, uint64_t initseq, uint32_t bound, uint32_t *out, int n)
{
    pcg32_random_t rng;
    pcg32_srandom_r(&rng, initstate, initseq);
    for (int i = 0; i < n; i++)
        out[i] = bound ? pcg32_boundedrand_r(&rng, bound) : pcg32_random_r(&rng);
}

void ref_set_st_weight(const int *cum, int n)
{
    for (int i = 0; i < n && i < MAX_STORAGE_TARGETS; i++)
        st_weight[i] = cum[i];
}

/* select_P would retry forever when no non-holder carries weight: report that
 * case as UINT64_MAX instead of calling it (fixtures never contain it). */
static int select_P_terminates(const FileInfo *fi, unsigned ntargets)
{
    if (sts_in_use(fi->locations) == (int)ntargets)
        return 1;
    for (unsigned t = 0; t < ntargets; t++)
        if (!TEST_BIT(fi->locations, t) && st_weight[t] - (t ? st_weight[t - 1] : 0) > 0)
            return 1;
    return 0;
}

uint64_t ref_select_P(const char *path, uint64_t locations, unsigned ntargets)
{
    FileInfo fi = {0, locations};
    if (!select_P_terminates(&fi, ntargets))
        return UINT64_MAX;
    select_P(path, &fi, ntargets);
    return fi.locations;
}

uint64_t ref_fill_in_missing_fields(uint64_t dst, uint64_t src)
{
    FileInfo d = {0, dst}, s = {0, src};
    fill_in_missing_fields(&d, &s);
    return d.locations;
}

void ref_fih_add_info(int64_t *timestamp, uint64_t *modified, uint64_t *deleted, int src, int64_t time, int rm)
{
    FatFileInfo fi = {*timestamp, *modified, *deleted};
    fih_add_info(&fi, src, time, rm);
    *timestamp = fi.timestamp;
    *modified = fi.modified;
    *deleted = fi.deleted;
}

/* gen/main.c:710-711: the worklist order, shuffle then qsort by total size
 * (this libc's qsort, as the reference links it). */
void ref_sort_order(const uint64_t *sizes, size_t n, uint64_t *idx)
{
    SizeIndex *a = malloc((n ? n : 1) * sizeof(SizeIndex));
    for (size_t i = 0; i < n; i++) {
        a[i].size = sizes[i];
        a[i].idx = i;
    }
    shuffle(a, n);
    qsort(a, n, sizeof(SizeIndex), cmp_entries);
    for (size_t i = 0; i < n; i++)
        idx[i] = a[i].idx;
    free(a);
}

/* gen/main.c:310 + 710-711 + 758: the coordinators' rounds.  paths[i]
 * (NUL-terminated, arrival order) goes to eater simple_hash % ntargets
 * (:310); each eater shuffles and qsorts its own SizeIndex array (:710-711);
 * the eaters broadcast one after another in rank order (:758), eater k =
 * storage target k here.  idx[] gets the indices in worklist order,
 * round_start[0..ntargets] the rounds' bounds. */
void ref_round_order(const char *const *paths, const uint64_t *sizes, size_t n, unsigned ntargets, uint64_t *idx,
                     size_t *round_start)
{
    SizeIndex *a = malloc((n ? n : 1) * sizeof(SizeIndex));
    size_t j = 0;
    for (unsigned k = 0; k < ntargets; k++) {
        round_start[k] = j;
        size_t m = 0;
        for (size_t i = 0; i < n; i++)
            if (simple_hash(paths[i], (int)strlen(paths[i])) % ntargets == k) {
                a[m].size = sizes[i];
                a[m].idx = i;
                m++;
            }
        shuffle(a, m);
        qsort(a, m, sizeof(SizeIndex), cmp_entries);
        for (size_t t = 0; t < m; t++)
            idx[j++] = a[t].idx;
    }
    round_start[ntargets] = j;
    free(a);
}

/* gen/main.c:772-788, one worklist item: the new FileInfo, merged with the
 * previous DB value when there is one (pdb_get), deleted holders dropped, P
 * chosen when invalid, NO_P when unchanged.  UINT64_MAX where select_P would
 * not terminate. */
uint64_t ref_plan_item(const char *s, int64_t timestamp, uint64_t modified, uint64_t deleted, int has_an_old_version,
                       int64_t old_timestamp, uint64_t old_locations, unsigned ntargets)
{
    FileInfo prev_fi = {old_timestamp, old_locations};
    FileInfo fi_, *fi = &fi_;
    fi->timestamp = timestamp;
    fi->locations = WITH_P(modified, NO_P);
    if (has_an_old_version)
        fill_in_missing_fields(fi, &prev_fi);
    fi->locations &= ~deleted;
    if (P_IS_INVALID(fi->locations)) {
        if (!select_P_terminates(fi, ntargets))
            return UINT64_MAX;
        select_P(s, fi, ntargets);
    }
    if (has_an_old_version && prev_fi.timestamp == fi->timestamp && prev_fi.locations == fi->locations)
        fi->locations = WITH_P(fi->locations, NO_P);
    return fi->locations;
}

int ref_store_weight(int dirfd)
{
    return get_store_weight(dirfd);
}

/* The same rounds with the eaters in MPI rank order (gen/main.c:758: round
 * r is broadcast by communicator rank r+1 = world rank 2r+1, the eater of
 * storage target round_st[r] = rank2st[2r+1] as ref_map_targets prints it,
 * gen/main.c:506-541); round_st NULL = target order (ref_round_order). */
void ref_round_order_ranked(const char *const *paths, const uint64_t *sizes, size_t n, unsigned ntargets,
                            const int *round_st, uint64_t *idx, size_t *round_start)
{
    SizeIndex *a = malloc((n ? n : 1) * sizeof(SizeIndex));
    size_t j = 0;
    for (unsigned r = 0; r < ntargets; r++) {
        const unsigned k = round_st ? (unsigned)round_st[r] : r;
        round_start[r] = j;
        size_t m = 0;
        for (size_t i = 0; i < n; i++)
            if (simple_hash(paths[i], (int)strlen(paths[i])) % ntargets == k) {
                a[m].size = sizes[i];
                a[m].idx = i;
                m++;
            }
        shuffle(a, m);
        qsort(a, m, sizeof(SizeIndex), cmp_entries);
        for (size_t t = 0; t < m; t++)
            idx[j++] = a[t].idx;
    }
    round_start[ntargets] = j;
    free(a);
}
