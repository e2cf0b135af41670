// haplofile.hpp — HPM / HPM2 / BENCH2 / BENCH3 genotype files (HaploFile.cpp:205-640).
#pragma once
#include <cstdint>
#include <string>
#include <vector>

namespace hmc {

struct FileData {
  int N = 0, L = 0;
  std::vector<int32_t> al;          // [N][2][L] symbols, -1 missing
  std::string types;                // per locus 'S' (character allele) or 'M' (integer)
  std::vector<std::string> ids;     // [N]
  std::vector<std::string> names;   // [L] marker names
  std::vector<int> pos;             // [L] marker positions
  int unphased = -1;                // GenoData::unphased_num (BENCH3: the parents); -1 = all N
};

// paths: PHASE/HPM/HPM2 one file; BENCH2 genotype + position file; BENCH3
// genotype + position + children file (HaploFile::getHaploFile, HaploFile.cpp:28-47).
bool read_geno_file(const std::string &format, const std::vector<std::string> &paths, FileData &d, std::string &err);
int geno_file_count(const std::string &format);  // HaploFile::getFileNameNum (HaploFile.cpp:13-26), 0 = unknown
bool write_geno_file(const std::string &format, const char *path, const char *path2, const FileData &d,
                     const std::vector<int32_t> &hap, std::string &err);

}  // namespace hmc
