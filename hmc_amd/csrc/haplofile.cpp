// haplofile.cpp — the genotype file formats of HaploFile besides PHASE
// (HaploFile.cpp:205-640), host C++.  Readers produce symbols per allele in
// the reference's conventions (single-character 'S' loci hold the character
// code, 'M' loci the integer, -1 = missing) plus ids, marker names and
// positions; writers emit the reference's output layout for a haplotype pair
// per individual.
//
//   HPM    header "Id [Status] [CONFIG_ID] name... [CONFIDENCE]", one haplotype
//          per line "id [fields] a1 a2 ...", integer alleles (0 = missing);
//          loci with at most two alleles become 'S' loci ('1'..'9', 'A'..'Z')
//   HPM2   the same with single-character alleles ('0' = missing, '1'..'9',
//          'A'..'Z' / 'a'..'z' = 10..35), converted as HPM's
//   BENCH2 genotype file (one haplotype per line: L characters, '0' missing,
//          '9' = the heterozygous placeholder, then "number 0 id") + position
//          file ("index name position")
//   BENCH3 BENCH2 + a children file in the same layout (HaploFile.cpp:446-484).
//          The children are appended as ordinary genotypes: setHaplotypes
//          leaves every genotype unphased (Genotype.cpp:40), so the EM resolves
//          them like the parents; only HaploComp stops at unphased_num = the
//          parents (HaploFile.cpp:475, HaploComp.cpp:40).
#include "haplofile.hpp"

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <set>

namespace hmc {

namespace {

const char *DELIM = " \t\r\n";

// Allele.cpp:55-79 readAllele
char *read_allele(char type, char *buf, int32_t &a) {
  buf += strspn(buf, DELIM);
  if (type == 'S') {
    a = (buf[0] == '-' || buf[0] == '?') ? -1 : (int32_t)(unsigned char)buf[0];
    if (buf[0]) buf++;
  } else {
    if (buf[0] == '-' || buf[0] == '?') {
      a = -1;
    } else {
      const int v = atoi(buf);
      a = v > 0 ? v : -1;
    }
    buf += strcspn(buf, DELIM);
  }
  return buf;
}

bool read_lines(const char *path, std::vector<std::string> &lines, std::string &err) {
  FILE *fp = fopen(path, "r");
  if (!fp) {
    err = std::string("Can not open file ") + path + "!";
    return false;
  }
  std::string cur;
  char buf[65536];
  while (fgets(buf, sizeof buf, fp)) {
    cur += buf;
    if (!cur.empty() && cur.back() == '\n') {
      lines.push_back(cur);
      cur.clear();
    }
  }
  if (!cur.empty()) lines.push_back(cur);
  fclose(fp);
  return true;
}

bool blank(const std::string &s) { return s.find_first_not_of(DELIM) == std::string::npos; }

// HaploFileHPM::alleleTypeM2S / S2M (HaploFile.cpp:253-264)
int32_t m2s(int32_t a) {
  if (a >= 1 && a <= 9) return a + '0';
  if (a >= 10 && a <= 35) return a + 'A' - 10;
  return a;
}
int32_t s2m(int32_t a) {
  if (a >= '1' && a <= '9') return a - '0';
  if (a >= 'A' && a <= 'Z') return a - 'A' + 10;
  if (a >= 'a' && a <= 'z') return a - 'a' + 10;
  return a;
}

// GenoData::checkAlleleSymbol's distinct non-missing symbols of locus k
int distinct_alleles(const FileData &d, int k) {
  std::set<int32_t> s;
  for (int i = 0; i < d.N; ++i)
    for (int h = 0; h < 2; ++h) {
      const int32_t a = d.al[((size_t)i * 2 + h) * d.L + k];
      if (a >= 0) s.insert(a);
    }
  return (int)s.size();
}

// HaploFileHPM::readGenoData + checkHeader + readHaplotype (HaploFile.cpp:205-251,
// 309-332, 345-387) and HaploFileHPM2::readHaplotype (:389-416)
bool read_hpm(const char *path, bool hpm2, FileData &d, std::string &err) {
  std::vector<std::string> lines;
  if (!read_lines(path, lines, err)) return false;
  if (lines.empty()) {
    err = "Not a valid HPM file!";
    return false;
  }
  static const std::set<std::string> fields{"Id", "Status", "CONFIG_ID", "CONFIDENCE"};
  std::vector<std::string> tok;
  {
    std::string h = lines[0];
    for (char *s = strtok(&h[0], DELIM); s; s = strtok(nullptr, DELIM)) tok.push_back(s);
  }
  if (tok.empty() || tok[0] != "Id") {
    err = "Not a valid HPM file!";
    return false;
  }
  size_t t = 1;
  int line_start = 1;
  while (t < tok.size() && fields.count(tok[t])) {
    ++line_start;
    ++t;
  }
  d.names.clear();
  while (t < tok.size() && !fields.count(tok[t])) d.names.push_back(tok[t++]);
  d.L = (int)d.names.size();
  const std::string types(d.L, hpm2 ? 'S' : 'M');
  std::vector<std::vector<int32_t>> haps;
  std::vector<std::string> hid;
  for (size_t ln = 1; ln < lines.size(); ++ln) {
    if (blank(lines[ln])) continue;
    std::string b = lines[ln];
    char *s = strtok(&b[0], DELIM);
    std::string id = s;
    for (int i = 1; i < line_start && s; ++i) s = strtok(nullptr, DELIM);
    if (!s) {
      err = "Incorrect haplotype data in line " + std::to_string(ln + 1) + "!";
      return false;
    }
    s += strlen(s) + 1;  // the alleles follow the last id field
    std::vector<int32_t> h(d.L);
    for (int k = 0; k < d.L; ++k) {
      if (!*s) {
        err = "Incorrect haplotype data in line " + std::to_string(ln + 1) + "!";
        return false;
      }
      s = read_allele(types[k], s, h[k]);
      if (hpm2) h[k] = h[k] == '0' ? -1 : s2m(h[k]);
    }
    haps.push_back(std::move(h));
    hid.push_back(id);
  }
  if (haps.size() % 2) {
    err = "Incorrect haplotype data in line " + std::to_string(haps.size() + 2) + "!";
    return false;
  }
  d.N = (int)haps.size() / 2;
  d.al.assign((size_t)d.N * 2 * d.L, -1);
  d.ids.assign(d.N, "");
  for (int i = 0; i < d.N; ++i) {
    d.ids[i] = hid[2 * i];
    for (int h = 0; h < 2; ++h) std::copy(haps[2 * i + h].begin(), haps[2 * i + h].end(), d.al.begin() + ((size_t)i * 2 + h) * d.L);
  }
  // loci with at most two alleles become SNP loci (HaploFile.cpp:238-247)
  d.types.assign(d.L, 'M');
  for (int k = 0; k < d.L; ++k)
    if (distinct_alleles(d, k) <= 2) {
      d.types[k] = 'S';
      for (size_t q = 0; q < (size_t)d.N * 2; ++q) {
        int32_t &a = d.al[q * d.L + k];
        if (a >= 0) a = m2s(a);
      }
    }
  d.pos.resize(d.L);
  for (int k = 0; k < d.L; ++k) d.pos[k] = k * 1000;  // GenoData::setGenotypeLen default
  return true;
}

// HaploFileBench::readHaploFile + readHaplotype (HaploFile.cpp:528-564, 605-624):
// one haplotype per line, appended to haps/hid; the heterozygous placeholder
// restarts at '1' in every file.
bool read_bench_haplos(const char *path, int L, std::vector<std::vector<int32_t>> &haps, std::vector<std::string> &hid,
                       std::string &err) {
  std::vector<std::string> lines;
  if (!read_lines(path, lines, err)) return false;
  const size_t before = haps.size();
  int het = 1;  // '9' = the heterozygous placeholder: '1' on the first haplotype, '2' on the second
  for (size_t ln = 0; ln < lines.size(); ++ln) {
    if (blank(lines[ln])) continue;
    const char *buf = lines[ln].c_str();
    buf += strspn(buf, DELIM);
    if ((int)strcspn(buf, DELIM) != L) {
      err = "Incorrect haplotype data in line " + std::to_string(ln + 1) + " of " + path + "!";
      return false;
    }
    std::vector<int32_t> h(L);
    for (int k = 0; k < L; ++k) {
      const char c = buf[k];
      h[k] = c == '0' ? -1 : (c == '9' ? '0' + het : (int32_t)(unsigned char)c);
    }
    const char *s = buf + L;
    for (int f = 0; f < 2; ++f) {  // skip the number and the 0
      s += strspn(s, DELIM);
      s += strcspn(s, DELIM);
    }
    s += strspn(s, DELIM);
    hid.push_back(std::string(s, strcspn(s, "\r\n")));
    haps.push_back(std::move(h));
    het = 3 - het;
  }
  if ((haps.size() - before) % 2) {
    err = "Incorrect haplotype data in line " + std::to_string(haps.size() - before + 2) + "!";
    return false;
  }
  return true;
}

// HaploFileBench::readGenoData / readPositionInfo (HaploFile.cpp:446-484, 566-588)
bool read_bench(const char *geno, const char *posinfo, const char *children, FileData &d, std::string &err) {
  std::vector<std::string> lines;
  if (!read_lines(geno, lines, err)) return false;
  if (lines.empty()) {
    err = "Invalid file type!";
    return false;
  }
  {
    const std::string &l0 = lines[0];
    const size_t b = l0.find_first_not_of(DELIM);
    d.L = b == std::string::npos ? 0 : (int)strcspn(l0.c_str() + b, DELIM);
  }
  d.types.assign(d.L, 'S');
  d.names.resize(d.L);
  d.pos.resize(d.L);
  for (int k = 0; k < d.L; ++k) {
    d.names[k] = "M" + std::to_string(k + 1);
    d.pos[k] = k * 1000;
  }
  std::vector<std::vector<int32_t>> haps;
  std::vector<std::string> hid;
  if (!read_bench_haplos(geno, d.L, haps, hid, err)) return false;
  const int parents = (int)haps.size() / 2;
  if (children && !read_bench_haplos(children, d.L, haps, hid, err)) return false;
  d.unphased = children ? parents : -1;  // setUnphasedNum(m_parents_num) (HaploFile.cpp:475)
  d.N = (int)haps.size() / 2;
  d.al.assign((size_t)d.N * 2 * d.L, -1);
  d.ids.assign(d.N, "");
  for (int i = 0; i < d.N; ++i) {
    d.ids[i] = hid[2 * i];
    for (int h = 0; h < 2; ++h) std::copy(haps[2 * i + h].begin(), haps[2 * i + h].end(), d.al.begin() + ((size_t)i * 2 + h) * d.L);
  }
  std::vector<std::string> pl;
  if (!read_lines(posinfo, pl, err)) return false;
  for (auto &l : pl) {
    std::string b = l;
    char *s = strtok(&b[0], DELIM);
    if (!s) continue;
    const int i = atoi(s);
    if (i >= 0 && i < d.L) {
      if ((s = strtok(nullptr, DELIM))) d.names[i] = s;
      if ((s = strtok(nullptr, DELIM))) d.pos[i] = atoi(s);
    }
  }
  return true;
}

}  // namespace

int geno_file_count(const std::string &format) {
  if (format == "PHASE" || format == "HPM" || format == "HPM2") return 1;
  if (format == "BENCH2") return 2;
  if (format == "BENCH3") return 3;
  return 0;
}

bool read_geno_file(const std::string &format, const std::vector<std::string> &paths, FileData &d, std::string &err) {
  const int need = geno_file_count(format);
  if (need == 0 || format == "PHASE") {
    err = "Unknown file format " + format;
    return false;
  }
  if ((int)paths.size() < need) {
    err = format + " needs " + std::to_string(need) + " file names";
    return false;
  }
  if (format == "HPM") return read_hpm(paths[0].c_str(), false, d, err);
  if (format == "HPM2") return read_hpm(paths[0].c_str(), true, d, err);
  return read_bench(paths[0].c_str(), paths[1].c_str(), format == "BENCH3" ? paths[2].c_str() : nullptr, d, err);
}

// HaploFileHPM(2)::writeGenoData + writeHaplotype (HaploFile.cpp:266-286,
// 334-343, 418-440) and HaploFileBench::writeGenoData + writePositionInfo
// (:486-505, 590-603), for the haplotype pairs hap[N][2][L] (symbols).
bool write_geno_file(const std::string &format, const char *path, const char *path2, const FileData &d,
                     const std::vector<int32_t> &hap, std::string &err) {
  const int N = d.N, L = d.L;
  FILE *fp = fopen(path, "w");
  if (!fp) {
    err = std::string("Can not open file ") + path + "!";
    return false;
  }
  if (format == "HPM" || format == "HPM2") {
    fprintf(fp, "Id\t");
    for (int k = 0; k < L; ++k) fprintf(fp, "%s ", d.names[k].c_str());
    fprintf(fp, "\n");
    for (int i = 0; i < N; ++i)
      for (int h = 0; h < 2; ++h) {
        fprintf(fp, "%s\t", d.ids[i].c_str());
        for (int k = 0; k < L; ++k) {
          int32_t a = hap[((size_t)i * 2 + h) * L + k];
          if (format == "HPM2") {  // every locus written as a character, '0' = missing
            if (a < 0) a = '0';
            else if (d.types[k] != 'S') a = m2s(a);
            fprintf(fp, "%c ", (char)a);
          } else if (d.types[k] == 'S') {
            fprintf(fp, "%c ", a < 0 ? '?' : (char)a);
          } else {
            fprintf(fp, "%d ", a);
          }
        }
        fprintf(fp, "\n");
      }
  } else if (format == "BENCH2" || format == "BENCH3") {
    for (int i = 0; i < N; ++i)
      for (int h = 0; h < 2; ++h) {
        for (int k = 0; k < L; ++k) {
          const int32_t a = hap[((size_t)i * 2 + h) * L + k];
          fputc(a < 0 ? '0' : (char)a, fp);
        }
        std::string id = d.ids[i];  // Haplotype::setID replaces spaces (Haplotype.h:26, Genotype.h:107-113)
        for (char &ch : id)
          if (ch == ' ') ch = '_';
        fprintf(fp, "   %d 0 %s\n", 2 * i + h, id.c_str());
      }
  } else {
    fclose(fp);
    err = "Unknown output format " + format;
    return false;
  }
  fclose(fp);
  if ((format == "BENCH2" || format == "BENCH3") && path2) {
    FILE *fq = fopen(path2, "w");
    if (!fq) {
      err = std::string("Can not open file ") + path2 + "!";
      return false;
    }
    for (int k = 0; k < L; ++k) fprintf(fq, " %d   %s   %d\n", k, d.names[k].c_str(), d.pos[k]);
    fclose(fq);
  }
  return true;
}

}  // namespace hmc
