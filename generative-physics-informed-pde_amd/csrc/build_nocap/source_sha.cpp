extern "C" const char* gpi_source_sha(void) { return "6065cb2b02928b2b47a1bce2d7a78306a4b5fbfc"; }
