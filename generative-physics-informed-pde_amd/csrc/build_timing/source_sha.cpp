extern "C" const char* gpi_source_sha(void) { return "a096d459f067b29796020156b6773f31239fbbf1"; }
