/* ORACLE / TEST INFRASTRUCTURE ONLY — local bundle adjustment restatement (placeholder; filled in later). */
#ifndef LBA_ORACLE_H
#define LBA_ORACLE_H
#endif
