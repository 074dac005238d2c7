extern "C" const char* gpi_source_sha(void) { return "ae07b18d8aee5e9b17510fe899521a0384fcd685"; }
