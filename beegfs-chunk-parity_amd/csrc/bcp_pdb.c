/*
 * bcp_pdb.c -- persistent chunk state: path -> FileInfo, iterated in key
 * order.  Replaces persistent_db.{c,h} (src/beegfs-raid5/common/
 * persistent_db.c:23-145), which wraps LevelDB -- absent from this image and
 * from the GPU box, so this is a self-contained store with the same
 * contract:
 *
 *   pdb_init(folder, version)  create-if-missing; a version stored under
 *                              "?db_version" must match (:51-75)
 *   pdb_set / pdb_del / pdb_get  16-byte FileInfo values (:85-125)
 *   pdb_iterate                bytewise key order (LevelDB's default
 *                              comparator), the version key skipped (:127-145)
 *
 * and LevelDB's write behaviour as the reference configures it
 * (write_options sync = 0): every update is appended to a log before the
 * call returns, durable against a process crash, not against power loss
 * unless bcp_pdb_sync() is called.
 *
 * Layout: <folder>/bcp_pdb.log =
 *   header  "BCPPDB01" u64 version
 *   records u8 op (1 set, 2 del) u8 0 u16 keylen key[keylen]
 *           [FileInfo, 16 B, set only] u32 FNV-1a of the preceding bytes
 * Open replays the log into a hash table; a torn or corrupt tail (a crash
 * mid-append) is cut at the last whole record, as LevelDB's log reader drops
 * a partial trailing block.  The log is rewritten with only live entries
 * when it holds more than twice as many records as live keys.
 *
 * Thread-safe: gen lanes (gen/main.c:146-149) update it concurrently.
 */
#define _GNU_SOURCE
#include <errno.h>
#include <fcntl.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>
#include <unistd.h>

#include "bcp_task.h"

#define PDB_MAGIC "BCPPDB01"
#define PDB_LOG "bcp_pdb.log"
#define PDB_VERSION_KEY "?db_version" /* persistent_db.c:13 */
#define OP_SET 1
#define OP_DEL 2

typedef struct {
    char *key;      /* NULL = never used */
    uint64_t hash;
    FileInfo fi;
    uint16_t keylen;
    uint8_t live;   /* 0 = tombstone (deleted) */
} slot_t;

struct bcp_pdb {
    pthread_mutex_t lock;
    char *dir;
    int fd;           /* log, O_APPEND */
    uint64_t version;
    slot_t *slots;
    size_t cap;       /* power of two */
    size_t used;      /* slots with a key (live or tombstone) */
    size_t live;
    size_t records;   /* records in the log */
};

static uint64_t fnv64(const void *p, size_t n)
{
    const unsigned char *b = p;
    uint64_t h = 0xcbf29ce484222325ULL;
    for (size_t i = 0; i < n; i++)
        h = (h ^ b[i]) * 0x100000001b3ULL;
    return h;
}

static uint32_t fnv32(const void *p, size_t n)
{
    const unsigned char *b = p;
    uint32_t h = 0x811c9dc5u;
    for (size_t i = 0; i < n; i++)
        h = (h ^ b[i]) * 0x01000193u;
    return h;
}

static int key_ok(const char *key, size_t keylen)
{
    if (!key || keylen == 0 || keylen > BCP_PDB_MAX_KEY)
        return 0;
    if (keylen == sizeof(PDB_VERSION_KEY) - 1 && !memcmp(key, PDB_VERSION_KEY, keylen))
        return 0; /* reserved (persistent_db.c:12-13) */
    return memchr(key, '\0', keylen) == NULL;
}

static slot_t *find_slot(const bcp_pdb *db, const char *key, size_t keylen, uint64_t h)
{
    size_t m = db->cap - 1;
    for (size_t i = h & m;; i = (i + 1) & m) {
        slot_t *s = &db->slots[i];
        if (!s->key)
            return s;
        if (s->hash == h && s->keylen == keylen && !memcmp(s->key, key, keylen))
            return s;
    }
}

static int grow(bcp_pdb *db)
{
    size_t ncap = db->cap ? db->cap : 1024;
    while (db->live * 2 + 16 > ncap / 2)
        ncap *= 2;
    slot_t *ns = calloc(ncap, sizeof(slot_t));
    if (!ns)
        return -ENOMEM;
    slot_t *old = db->slots;
    size_t ocap = db->cap;
    db->slots = ns;
    db->cap = ncap;
    db->used = 0;
    for (size_t i = 0; i < ocap; i++) {
        if (!old[i].key)
            continue;
        if (!old[i].live) {
            free(old[i].key); /* drop tombstones */
            continue;
        }
        slot_t *s = find_slot(db, old[i].key, old[i].keylen, old[i].hash);
        *s = old[i];
        db->used++;
    }
    free(old);
    return 0;
}

/* In-memory apply (no log write). */
static int apply(bcp_pdb *db, int op, const char *key, size_t keylen, const FileInfo *fi)
{
    if (op == OP_SET && (db->used + 1) * 10 > db->cap * 7) {
        int rc = grow(db);
        if (rc)
            return rc;
    }
    const uint64_t h = fnv64(key, keylen);
    slot_t *s = find_slot(db, key, keylen, h);
    if (op == OP_SET) {
        if (!s->key) {
            s->key = malloc(keylen);
            if (!s->key)
                return -ENOMEM;
            memcpy(s->key, key, keylen);
            s->keylen = (uint16_t)keylen;
            s->hash = h;
            db->used++;
        }
        if (!s->live)
            db->live++;
        s->live = 1;
        s->fi = *fi;
    } else if (s->key && s->live) {
        s->live = 0;
        db->live--;
    }
    return 0;
}

static size_t encode(unsigned char *buf, int op, const char *key, size_t keylen, const FileInfo *fi)
{
    size_t n = 0;
    buf[n++] = (unsigned char)op;
    buf[n++] = 0;
    const uint16_t kl = (uint16_t)keylen;
    memcpy(buf + n, &kl, 2);
    n += 2;
    memcpy(buf + n, key, keylen);
    n += keylen;
    if (op == OP_SET) {
        memcpy(buf + n, fi, sizeof(FileInfo));
        n += sizeof(FileInfo);
    }
    const uint32_t c = fnv32(buf, n);
    memcpy(buf + n, &c, 4);
    return n + 4;
}

static int write_all(int fd, const void *p, size_t n)
{
    const char *b = p;
    while (n) {
        ssize_t w = write(fd, b, n);
        if (w < 0) {
            if (errno == EINTR)
                continue;
            return -errno;
        }
        b += w;
        n -= (size_t)w;
    }
    return 0;
}

static int append(bcp_pdb *db, int op, const char *key, size_t keylen, const FileInfo *fi)
{
    unsigned char buf[8 + BCP_PDB_MAX_KEY + sizeof(FileInfo) + 4];
    const size_t n = encode(buf, op, key, keylen, fi);
    int rc = write_all(db->fd, buf, n); /* one write: O_APPEND keeps records whole */
    if (!rc)
        db->records++;
    return rc;
}

/* Replay the log; returns the offset after the last whole record. */
static int replay(bcp_pdb *db, const unsigned char *p, size_t size, size_t *good)
{
    size_t off = 16;
    while (off + 8 <= size) {
        const int op = p[off];
        uint16_t kl;
        memcpy(&kl, p + off + 2, 2);
        if ((op != OP_SET && op != OP_DEL) || p[off + 1] != 0 || kl == 0 || kl > BCP_PDB_MAX_KEY)
            break;
        const size_t body = 4 + (size_t)kl + (op == OP_SET ? sizeof(FileInfo) : 0);
        if (off + body + 4 > size)
            break;
        uint32_t c;
        memcpy(&c, p + off + body, 4);
        if (c != fnv32(p + off, body))
            break;
        FileInfo fi = {0, 0};
        if (op == OP_SET)
            memcpy(&fi, p + off + 4 + kl, sizeof(FileInfo));
        int rc = apply(db, op, (const char *)p + off + 4, kl, &fi);
        if (rc)
            return rc;
        db->records++;
        off += body + 4;
    }
    *good = off;
    return 0;
}

static int cmp_slot(const void *a, const void *b)
{
    const slot_t *x = *(slot_t *const *)a, *y = *(slot_t *const *)b;
    const size_t n = x->keylen < y->keylen ? x->keylen : y->keylen;
    const int c = memcmp(x->key, y->key, n); /* bytewise, unsigned */
    if (c)
        return c;
    return (x->keylen > y->keylen) - (x->keylen < y->keylen);
}

/* Live slots sorted by key (caller holds the lock; free the array). */
static slot_t **sorted_live(const bcp_pdb *db, size_t *n)
{
    slot_t **v = malloc((db->live ? db->live : 1) * sizeof(slot_t *));
    if (!v)
        return NULL;
    size_t k = 0;
    for (size_t i = 0; i < db->cap; i++)
        if (db->slots[i].key && db->slots[i].live)
            v[k++] = &db->slots[i];
    qsort(v, k, sizeof(slot_t *), cmp_slot);
    *n = k;
    return v;
}

static int path_in(const bcp_pdb *db, const char *name, char *out, size_t cap)
{
    int n = snprintf(out, cap, "%s/%s", db->dir, name);
    return (n < 0 || (size_t)n >= cap) ? -ENAMETOOLONG : 0;
}

static int write_header(int fd, uint64_t version)
{
    unsigned char h[16];
    memcpy(h, PDB_MAGIC, 8);
    memcpy(h + 8, &version, 8);
    return write_all(fd, h, 16);
}

/* Rewrite the log with the live entries only (caller holds the lock). */
static int compact(bcp_pdb *db)
{
    char tmp[4096], fin[4096];
    int rc = path_in(db, PDB_LOG ".tmp", tmp, sizeof(tmp));
    if (!rc)
        rc = path_in(db, PDB_LOG, fin, sizeof(fin));
    if (rc)
        return rc;
    size_t n = 0;
    slot_t **v = sorted_live(db, &n);
    if (!v)
        return -ENOMEM;
    int fd = open(tmp, O_WRONLY | O_CREAT | O_TRUNC | O_CLOEXEC, 0600);
    if (fd < 0) {
        free(v);
        return -errno;
    }
    rc = write_header(fd, db->version);
    /* buffer records: one write per ~1 MiB */
    size_t cap = 1 << 20, len = 0;
    unsigned char *buf = rc ? NULL : malloc(cap + 512);
    if (!rc && !buf)
        rc = -ENOMEM;
    for (size_t i = 0; !rc && i < n; i++) {
        len += encode(buf + len, OP_SET, v[i]->key, v[i]->keylen, &v[i]->fi);
        if (len >= cap) {
            rc = write_all(fd, buf, len);
            len = 0;
        }
    }
    if (!rc && len)
        rc = write_all(fd, buf, len);
    free(buf);
    free(v);
    if (!rc && fsync(fd) != 0)
        rc = -errno;
    close(fd);
    if (!rc && rename(tmp, fin) != 0)
        rc = -errno;
    if (rc) {
        unlink(tmp);
        return rc;
    }
    int nfd = open(fin, O_WRONLY | O_APPEND | O_CLOEXEC);
    if (nfd < 0)
        return -errno;
    close(db->fd);
    db->fd = nfd;
    db->records = n;
    return 0;
}

int bcp_pdb_open(const char *folder, uint64_t expected_version, bcp_pdb **out)
{
    if (!folder || !out)
        return -EINVAL;
    *out = NULL;
    if (mkdir(folder, 0700) != 0 && errno != EEXIST)
        return -errno;
    bcp_pdb *db = calloc(1, sizeof(*db));
    if (!db)
        return -ENOMEM;
    pthread_mutex_init(&db->lock, NULL);
    db->fd = -1;
    db->dir = strdup(folder);
    int rc = db->dir ? grow(db) : -ENOMEM;
    char path[4096];
    if (!rc)
        rc = path_in(db, PDB_LOG, path, sizeof(path));
    int fd = -1;
    if (!rc) {
        fd = open(path, O_RDWR | O_CREAT | O_CLOEXEC, 0600);
        if (fd < 0)
            rc = -errno;
    }
    struct stat st;
    if (!rc && fstat(fd, &st) != 0)
        rc = -errno;
    if (!rc && st.st_size == 0) {
        /* new database: record the version (persistent_db.c:65-71) */
        db->version = expected_version;
        rc = write_header(fd, expected_version);
    } else if (!rc) {
        size_t size = (size_t)st.st_size;
        unsigned char *p = malloc(size);
        if (!p)
            rc = -ENOMEM;
        size_t got = 0;
        while (!rc && got < size) {
            ssize_t r = pread(fd, p + got, size - got, (off_t)got);
            if (r < 0 && errno == EINTR)
                continue;
            if (r <= 0)
                rc = r < 0 ? -errno : -EIO;
            else
                got += (size_t)r;
        }
        if (!rc && (size < 16 || memcmp(p, PDB_MAGIC, 8) != 0))
            rc = -EPROTO; /* "Corrupt version field in database" */
        if (!rc) {
            memcpy(&db->version, p + 8, 8);
            if (db->version != expected_version)
                rc = -EPROTO; /* "Incompatible DB (found: %lu, expected: %lu)" */
        }
        size_t good = 16;
        if (!rc)
            rc = replay(db, p, size, &good);
        free(p);
        if (!rc && good < size && ftruncate(fd, (off_t)good) != 0)
            rc = -errno; /* drop a torn tail */
    }
    if (fd >= 0)
        close(fd);
    if (!rc) {
        db->fd = open(path, O_WRONLY | O_APPEND | O_CLOEXEC);
        if (db->fd < 0)
            rc = -errno;
    }
    if (!rc && db->records > 2 * db->live + 4096)
        rc = compact(db);
    if (rc) {
        bcp_pdb_close(db);
        return rc;
    }
    *out = db;
    return 0;
}

int bcp_pdb_close(bcp_pdb *db)
{
    if (!db)
        return -EINVAL;
    int rc = 0;
    pthread_mutex_lock(&db->lock);
    if (db->fd >= 0 && db->records > 2 * db->live + 4096)
        rc = compact(db);
    if (db->fd >= 0)
        close(db->fd);
    pthread_mutex_unlock(&db->lock);
    for (size_t i = 0; i < db->cap; i++)
        free(db->slots[i].key);
    free(db->slots);
    free(db->dir);
    pthread_mutex_destroy(&db->lock);
    free(db);
    return rc;
}

int bcp_pdb_set(bcp_pdb *db, const char *key, size_t keylen, const FileInfo *val)
{
    if (!db || !val || !key_ok(key, keylen))
        return -EINVAL;
    pthread_mutex_lock(&db->lock);
    int rc = append(db, OP_SET, key, keylen, val);
    if (!rc)
        rc = apply(db, OP_SET, key, keylen, val);
    pthread_mutex_unlock(&db->lock);
    return rc;
}

int bcp_pdb_del(bcp_pdb *db, const char *key, size_t keylen)
{
    if (!db || !key_ok(key, keylen))
        return -EINVAL;
    pthread_mutex_lock(&db->lock);
    int rc = append(db, OP_DEL, key, keylen, NULL);
    if (!rc)
        rc = apply(db, OP_DEL, key, keylen, NULL);
    pthread_mutex_unlock(&db->lock);
    return rc;
}

int bcp_pdb_get(bcp_pdb *db, const char *key, size_t keylen, FileInfo *val)
{
    if (!db || !val || !key_ok(key, keylen))
        return -EINVAL;
    pthread_mutex_lock(&db->lock);
    slot_t *s = find_slot(db, key, keylen, fnv64(key, keylen));
    int found = s->key && s->live;
    if (found)
        *val = s->fi;
    pthread_mutex_unlock(&db->lock);
    return found;
}

size_t bcp_pdb_count(bcp_pdb *db)
{
    if (!db)
        return 0;
    pthread_mutex_lock(&db->lock);
    size_t n = db->live;
    pthread_mutex_unlock(&db->lock);
    return n;
}

int bcp_pdb_sync(bcp_pdb *db)
{
    if (!db)
        return -EINVAL;
    pthread_mutex_lock(&db->lock);
    int rc = fsync(db->fd) == 0 ? 0 : -errno;
    pthread_mutex_unlock(&db->lock);
    return rc;
}

int bcp_pdb_items(bcp_pdb *db, bcp_work_item **items, size_t *nitems)
{
    if (!db || !items || !nitems)
        return -EINVAL;
    *items = NULL;
    *nitems = 0;
    pthread_mutex_lock(&db->lock);
    size_t n = 0;
    slot_t **v = sorted_live(db, &n);
    size_t keybytes = 0;
    for (size_t i = 0; v && i < n; i++)
        keybytes += v[i]->keylen + 1u;
    /* one block: items then NUL-terminated keys, freed with bcp_pdb_items_free */
    bcp_work_item *it = v ? malloc(n * sizeof(bcp_work_item) + keybytes + 1) : NULL;
    if (!it) {
        pthread_mutex_unlock(&db->lock);
        free(v);
        return -ENOMEM;
    }
    char *kp = (char *)(it + n);
    for (size_t i = 0; i < n; i++) {
        memcpy(kp, v[i]->key, v[i]->keylen);
        kp[v[i]->keylen] = '\0';
        it[i].path = kp;
        it[i].fi = v[i]->fi;
        kp += v[i]->keylen + 1u;
    }
    pthread_mutex_unlock(&db->lock);
    free(v);
    *items = it;
    *nitems = n;
    return 0;
}

void bcp_pdb_items_free(bcp_work_item *items)
{
    free(items);
}

int bcp_pdb_iterate(bcp_pdb *db, bcp_pdb_visit_fn fn, void *ctx)
{
    if (!db || !fn)
        return -EINVAL;
    bcp_work_item *it;
    size_t n;
    int rc = bcp_pdb_items(db, &it, &n); /* snapshot: fn may update the DB */
    if (rc)
        return rc;
    for (size_t i = 0; i < n; i++)
        if (fn(it[i].path, strlen(it[i].path), &it[i].fi, ctx))
            break; /* is_done (persistent_db.c:133-141) */
    bcp_pdb_items_free(it);
    return 0;
}
