    /* (end of the streamed reference code) */
    printf("st_ids");
    for (int i = 0; i < ntargets; i++)
        printf(" %d", last_run.targetIDs[i].id);
    printf("\nst2rank");
    for (int i = 0; i < ntargets; i++)
        printf(" %d", st2rank[i]);
    printf("\nround_st");
    for (int r = 0; r < ntargets; r++)
        printf(" %d", rank2st[2 * r + 1]);
    printf("\n");
}

int main(int argc, char **argv)
{
    int a = 1, prev[MAX_STORAGE_TARGETS], ids[MAX_STORAGE_TARGETS];
    if (argc < 3)
        return 2;
    const int nprev = atoi(argv[a++]);
    if (nprev < 0 || nprev > MAX_STORAGE_TARGETS || argc < a + nprev + 1)
        return 2;
    for (int i = 0; i < nprev; i++)
        prev[i] = atoi(argv[a++]);
    const int ntargets = atoi(argv[a++]);
    if (ntargets < 1 || ntargets > MAX_STORAGE_TARGETS || argc != a + ntargets)
        return 2;
    for (int r = 0; r < ntargets; r++)
        ids[r] = atoi(argv[a++]);
    run_map(nprev, prev, ntargets, ids);
    return 0;
}
